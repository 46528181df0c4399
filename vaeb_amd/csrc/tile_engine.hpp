// tile_engine.hpp -- fp32 MFMA tile engine for gfx950 (CDNA4).
//
// Every contraction of the SGVB step (VAEB.py:245-265 forward, the T.grad backward of
// VAEB.py:397) is C[M x N] = A[M x K] * B[K x N] with small, awkward shapes (M = batch
// rows = 100, K as small as Z = 20, N as small as Z).  At these sizes every phase is
// latency-bound, so the engine is built to put a wave's whole K share in flight at once:
//
//  * one wave owns a 16x16 output tile and runs v_mfma_f32_16x16x4_f32 (exact f32,
//    64 FLOP/clk/SIMD = the f32 peak of the chip) over its K-slice;
//  * a workgroup holds WM x WN tiles x KS K-slices (4 or 8 waves); K-slices are summed
//    through LDS before the fused epilogue;
//  * a wave loads GCH chunks (16 k each) into registers before its first MFMA -- one
//    memory round trip per group instead of one per chunk;
//  * loads are raw buffer loads (32-bit offsets, out-of-range reads return 0), so a
//    masked element costs one offset select and the load streams stay branch-free.
//
// Operand feeding (per lane l, i = l & 15, q = l >> 4, chunk c of 16 k-values): the
// MFMA's k-group q is fed k = 16c + 4q + s at step s = 0..3, so each lane needs FOUR
// CONSECUTIVE k at its fixed row (A) / column (B): one 16-byte load when the operand is
// K-contiguous, four coalesced scalar loads when it is M/N-contiguous.
// C/D mapping of 16x16x4 f32: col = l & 15, row = 4*(l >> 4) + r  (r = 0..3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Diagnostics: wave 0 of each workgroup records a 100 MHz timestamp in slot `slot`.
// Compiled in only with -DVAEB_TIMELINE (the `tl` library variant, __graft_entry__
// .build_variant): in the product build the stamp branches are dead code, so no kernel
// starts with a dependent load of its debug pointer ahead of its operand loads.
#ifdef VAEB_TIMELINE
#define VAEB_DBG_ON(p) ((p) != nullptr)
#else
#define VAEB_DBG_ON(p) false
#endif
#define VAEB_STAMP(A, slot)                                                               \
    do {                                                                                  \
        if (VAEB_DBG_ON((A).dbg) && threadIdx.x == 0)                                     \
            (A).dbg[(blockIdx.x + (uint64_t)blockIdx.y * gridDim.x) * 8 + (slot)] =       \
                __builtin_amdgcn_s_memrealtime();                                         \
    } while (0)

// ... at an explicit (logical) workgroup index, for fused grids whose parts stamp by
// logical id so their slots do not collide.
#define VAEB_STAMP_AT(A, idx, slot)                                                       \
    do {                                                                                  \
        if (VAEB_DBG_ON((A).dbg) && threadIdx.x == 0)                                     \
            (A).dbg[(uint64_t)(idx) * 8 + (slot)] = __builtin_amdgcn_s_memrealtime();     \
    } while (0)

// Diagnostics variant that first drains this wave's outstanding vector-memory operations,
// so the stamp marks when its loads have actually landed (debug launches only).
#define VAEB_STAMP_SYNC(A, slot)                                                          \
    do {                                                                                  \
        if (VAEB_DBG_ON((A).dbg)) {                                                       \
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                              \
            if (threadIdx.x == 0)                                                         \
                (A).dbg[(blockIdx.x + (uint64_t)blockIdx.y * gridDim.x) * 8 + (slot)] =   \
                    __builtin_amdgcn_s_memrealtime();                                     \
        }                                                                                 \
    } while (0)

namespace vaeb {

// Device control block (vaeb_hip.hip: ictl): [cursor, cur_batch, next, order[kOrderCap]].
// `next` = order[cursor] is kept by whoever advances the cursor (the step's last launch;
// upload_order for a fresh order), so the next step's encoder resolves its input rows
// with ONE dependent load instead of the cursor -> order[cursor] chain.  The head words
// and the order are contiguous, so a fresh order is one upload.
constexpr int kOrderCap = 1 << 20;
constexpr int kCtlNext = 2;    // offset of `next` from the cursor
constexpr int kCtlOrder = 3;   // offset of order[0]

// A control word that no workgroup of this launch writes (cursor / next / cur_batch, all
// written by earlier launches): read through the constant address space, i.e. a scalar
// load counted by lgkmcnt, so the wait for it does not drain the vector loads issued
// around it (a vector load + readfirstlane made hipcc wait vmcnt(0) before the first
// operand load of the launch could even be issued).
DEV int ld_launch_const(const int* p) {
    typedef const __attribute__((address_space(4))) int cint;
    return *(cint*)(uintptr_t)p;
}

DEV f32x4 zero4() { f32x4 z = {0.f, 0.f, 0.f, 0.f}; return z; }

// XCD-aware block order (guide T1): the dispatcher deals linear workgroup ids round-robin
// over the 8 XCDs (id % 8 labels the blocks that share one L2), so remap them to give
// each XCD one contiguous run of logical ids -- blocks that share an operand panel (the
// row blocks of one weight-column tile) then share that XCD's L2 instead of fetching
// the panel once per XCD.  Bijective for any n; a speed choice only (the kernels are
// placement independent).
DEV int xcd_remap(int b, int n) {
    if (n < 16) return b;
    const int xcd = b & 7, q = n >> 3, r = n & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// ------------------------------------------------------------------ buffer operands
// Every operand fetch is a raw buffer load through a 128-bit descriptor built from
// wave-uniform kernel arguments: a 32-bit per-lane byte offset, and the hardware range
// check returns 0 for an offset >= num_records.  Masking an element is therefore one
// select of its offset to kOOB -- no 64-bit address arithmetic and no select on the
// loaded value, which keeps the load streams short and lets them all issue before the
// first wait (the flat-pointer form of this code serialised behind vmcnt(0)).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0x80000000u;  // every buffer here is < 2 GiB

// The descriptor inputs go through readfirstlane so the compiler can PROVE them
// wave-uniform (otherwise it wraps every buffer op in a waterfall loop; guide T20).
DEV rsrc_t mkbuf(const void* p, int64_t nbytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int n = __builtin_amdgcn_readfirstlane((int)(nbytes < 0x7FFFFFF0ll ? nbytes : 0x7FFFFFF0ll));
    void* base = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, n, 0x00020000);
}
DEV float bld(rsrc_t b, uint32_t off) { return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b, off, 0, 0)); }
DEV f32x4 bld4(rsrc_t b, uint32_t off) { return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(b, off, 0, 0)); }
// AUX = 16: sc1 (loads bypass L1; stores write through) -- the in-launch hand-off form
template <int AUX>
DEV float bldx(rsrc_t b, uint32_t off) { return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b, off, 0, AUX)); }
template <int AUX>
DEV f32x4 bld4x(rsrc_t b, uint32_t off) { return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(b, off, 0, AUX)); }
template <int AUX>
DEV void bst4x(rsrc_t b, uint32_t off, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v), b, off, 0, AUX);
}
typedef __attribute__((address_space(1))) int gint;   // global int (agent-scope atomics)
DEV void bst(rsrc_t b, uint32_t off, float v) { __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), b, off, 0, 0); }
// Optimizer stores (theta', accumulator) are written through (sc1): the next launch reads
// them from other XCDs anyway, and a launch that ends with megabytes of dirty L2 lines pays
// their write-back at its boundary.  MNIST-20: dW2 9.5 -> 9.1 us, dW3 | dW45 7.5 -> 7.1 us
// (nt instead: no change).
constexpr int kStWT = 16;
DEV void bst_opt(rsrc_t b, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), b, off, 0, kStWT);
}

DEV bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// K-contiguous operand: element (r, k) at [r * ld + k]; r >= rlim or k >= klim read 0.
// vec: ld % 4 == 0, klim % 4 == 0 and a 16-byte aligned base (a float4 at k % 4 == 0 is
// then wholly in or wholly out of range).
DEV f32x4 kc4(rsrc_t b, int ld, int r, int k, int rlim, int klim, bool vec) {
    const bool rok = r < rlim;
    const uint32_t base = (uint32_t)(r * ld + k) * 4u;
    if (vec) return bld4(b, (rok && k < klim) ? base : kOOB);
    f32x4 v;
    v.x = bld(b, (rok && k + 0 < klim) ? base + 0 : kOOB);
    v.y = bld(b, (rok && k + 1 < klim) ? base + 4 : kOOB);
    v.z = bld(b, (rok && k + 2 < klim) ? base + 8 : kOOB);
    v.w = bld(b, (rok && k + 3 < klim) ? base + 12 : kOOB);
    return v;
}

// kc4 with a cache-policy operand (AUX 16: the sc1 loads of an in-launch hand-off)
template <int AUX>
DEV f32x4 kc4x(rsrc_t b, int ld, int r, int k, int rlim, int klim, bool vec) {
    const bool rok = r < rlim;
    const uint32_t base = (uint32_t)(r * ld + k) * 4u;
    if (vec) return bld4x<AUX>(b, (rok && k < klim) ? base : kOOB);
    f32x4 v;
    v.x = bldx<AUX>(b, (rok && k + 0 < klim) ? base + 0 : kOOB);
    v.y = bldx<AUX>(b, (rok && k + 1 < klim) ? base + 4 : kOOB);
    v.z = bldx<AUX>(b, (rok && k + 2 < klim) ? base + 8 : kOOB);
    v.w = bldx<AUX>(b, (rok && k + 3 < klim) ? base + 12 : kOOB);
    return v;
}

// M/N-contiguous operand: element (r, k) at [k * ld + r].
DEV f32x4 mc4(rsrc_t b, int ld, int r, int k, int rlim, int klim) {
    const bool rok = r < rlim;
    const uint32_t base = (uint32_t)(k * ld + r) * 4u;
    const uint32_t st = (uint32_t)ld * 4u;
    f32x4 v;
    v.x = bld(b, (rok && k + 0 < klim) ? base : kOOB);
    v.y = bld(b, (rok && k + 1 < klim) ? base + st : kOOB);
    v.z = bld(b, (rok && k + 2 < klim) ? base + 2 * st : kOOB);
    v.w = bld(b, (rok && k + 3 < klim) ? base + 3 * st : kOOB);
    return v;
}

DEV f32x4 mfma4(f32x4 a, f32x4 b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
    return c;
}

// One DPP lane move within a 16-lane row (all rows and banks enabled).
template <int CTRL>
DEV float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// Sum over the 16 lanes that share l >> 4 (one output row group of the C/D map), every lane
// ending with the same value: quad_perm [1,0,3,2] and [2,3,0,1] (quad sums), row_half_mirror
// (lane i <- 7 - i: the other quad of the half-row), row_mirror (lane i <- 15 - i: the other
// half).  Four VALU-latency DPP adds instead of four ds_bpermute round trips through the LDS
// unit (~100 cycles each with their waits: they dominated a single wave's epilogue rows).
DEV float sum16(float v) {
    v += dppf<0xB1>(v);
    v += dppf<0x4E>(v);
    v += dppf<0x141>(v);
    v += dppf<0x140>(v);
    return v;
}

// The wave-level main loop: accumulate NB tiles that share the A operand, over the
// chunks c = kslice, kslice + KS, ... < ceil(K/16), GCH chunks per memory round trip.
// P must provide:  f32x4 a4(int m, int k) const;  f32x4 b4(int n, int k, int which) const;
template <int NB, int KS, int GCH, class P>
DEV void wave_mainloop(const P& p, int m, int n, int K, int kslice, f32x4 (&acc)[NB]) {
    const int lane = threadIdx.x & 63;
    const int kq = 4 * (lane >> 4);
    const int nch = (K + 15) >> 4;
    for (int c0 = kslice; c0 < nch; c0 += GCH * KS) {
        f32x4 a[GCH], b[GCH][NB];
#pragma unroll
        for (int u = 0; u < GCH; ++u) {
            const int k = (c0 + u * KS) * 16 + kq;  // k >= K: the loaders return zeros
            a[u] = p.a4(m, k);
#pragma unroll
            for (int w = 0; w < NB; ++w) b[u][w] = p.b4(n, k, w);
        }
#pragma unroll
        for (int u = 0; u < GCH; ++u)
#pragma unroll
            for (int w = 0; w < NB; ++w) acc[w] = mfma4(a[u], b[u][w], acc[w]);
    }
}

// Sum the KS K-slice partials of each tile through LDS; afterwards the ks == 0 wave of
// each tile holds the total.  Returns false for the other waves.
template <int NW, int KS, int NB>
DEV bool ks_reduce(f32x4 (&acc)[NB], int wave, int ks) {
    if constexpr (KS > 1) {
        __shared__ f32x4 red[NW][NB][64];
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int w = 0; w < NB; ++w) red[wave][w][lane] = acc[w];
        __syncthreads();
        if (ks != 0) return false;
#pragma unroll
        for (int s = 1; s < KS; ++s)
#pragma unroll
            for (int w = 0; w < NB; ++w) acc[w] += red[wave + s][w][lane];
    }
    return true;
}

// Generic tile kernel.  Grid: x = M tiles / WM, y = N tiles / WN; WM*WN*KS waves.
// P also provides  int M, N, K;  void prepare();
//                  Pre prefetch(int m0, int n0) const;   (epilogue operands, issued
//                      before the main loop so they ride the same memory round trip)
//                  void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre&) const;
// One output tile (bx, by) of phase P; the standalone kernel and the horizontally fused
// launches (phase tiles + weight-gradient tiles in one grid) share this body.
template <int WM, int WN, int KS, int NB, int GCH, class P>
DEV void tile_body(P& p, int bx, int by) {
    constexpr int NW = WM * WN * KS;
    const int lin = bx + by * (int)gridDim.x;  // 1-D fused grids have gridDim.y == 1 and by == 0
    if (VAEB_DBG_ON(p.a.dbg) && threadIdx.x == 0) p.a.dbg[(uint64_t)lin * 8 + 6] = __builtin_amdgcn_s_memtime();
    p.prepare();
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int ks = wave % KS;
    const int t = wave / KS;
    const int m0 = (bx * WM + t / WN) * 16;
    const int n0 = (by * WN + t % WN) * 16;
    f32x4 acc[NB];
#pragma unroll
    for (int w = 0; w < NB; ++w) acc[w] = zero4();
    typename P::Pre pre{};
    if (ks == 0) pre = p.prefetch(m0, n0);
    if (m0 < p.M && n0 < p.N) wave_mainloop<NB, KS, GCH>(p, m0 + (lane & 15), n0 + (lane & 15), p.K, ks, acc);
    VAEB_STAMP(p.a, 1);
    if (!ks_reduce<NW, KS, NB>(acc, wave, ks)) return;
    VAEB_STAMP(p.a, 2);
    if (m0 >= p.M || n0 >= p.N) return;
    p.epilogue(m0, n0, acc, pre);
    VAEB_STAMP(p.a, 3);
    if (VAEB_DBG_ON(p.a.dbg) && threadIdx.x == 0) p.a.dbg[(uint64_t)lin * 8 + 7] = __builtin_amdgcn_s_memtime();
}

template <int WM, int WN, int KS, int NB, int GCH, class P>
__global__ __launch_bounds__(64 * WM * WN * KS) void tile_kernel(P p0) {
    P p = p0;
    VAEB_STAMP(p.a, 0);
    tile_body<WM, WN, KS, NB, GCH, P>(p, blockIdx.x, blockIdx.y);
}

// ------------------------------------------------------------------ Philox4x32-10
DEV void philox4x32(uint32_t (&ctr)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ ctr[1] ^ k0;
        const uint32_t n2 = hi0 ^ ctr[3] ^ k1;
        ctr[0] = n0; ctr[1] = lo1; ctr[2] = n2; ctr[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// ------------------------------------------------------------ fast transcendentals
// Every phase here is latency-bound with 8-16 waves per CU, so the libm (ocml) forms --
// range reduction, special-case branches, IEEE division -- made the element-wise stages
// VALU-bound (the latent middle took 3 us).  These use the hardware approximations
// (v_exp_f32 / v_log_f32 / v_rcp_f32 / v_sqrt_f32 / v_cos_f32, ~1 ulp each); the
// resulting differences (~1e-6 relative) sit far inside the parity tolerance (1e-4).
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
DEV float fexp(float x) { return __builtin_amdgcn_exp2f(x * kLog2e); }
DEV float flog(float x) { return __builtin_amdgcn_logf(x) * kLn2; }
DEV float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
// tanh: odd; 1 - 2 / (e^{2|x|} + 1) away from 0, Taylor below 1/16 (no cancellation)
DEV float ftanh(float x) {
    const float ax = fabsf(x);
    const float x2 = ax * ax;
    const float small = ax * (1.f + x2 * (-1.f / 3.f + x2 * (2.f / 15.f)));
    const float big = 1.f - 2.f * frcp(fexp(2.f * ax) + 1.f);
    return copysignf(ax < 0.0625f ? small : big, x);
}
DEV float softplusf(float a) { return fmaxf(a, 0.f) + flog(1.f + fexp(-fabsf(a))); }
DEV float sigmoidf(float a) { return frcp(1.f + fexp(-a)); }
// sigmoid(a) and softplus(a) from ONE exponential: t = e^{-|a|}, sigmoid = 1/(1+t) (a >= 0)
// or t/(1+t), softplus = max(a, 0) + log(1 + t)  (the Bernoulli decoder's y and BCE).
DEV void sigmoid_softplus(float a, float& y, float& sp) {
    const float t = fexp(-fabsf(a));
    const float d = 1.f + t;
    const float r = frcp(d);
    y = a >= 0.f ? r : t * r;
    sp = fmaxf(a, 0.f) + flog(d);
}

// Counter words 2-3 of a draw: the step, the validation flag (domain bit 0) in bit 63 and
// the reconstruction sample stream (domain >> 1, VAEB.py:279-280) in bits 40..62.
DEV uint64_t philox_c23(int64_t step, uint32_t domain) {
    return (uint64_t)step ^ ((uint64_t)(domain & 1u) << 63) ^ ((uint64_t)(domain >> 1) << 40);
}

// One standard normal for the 128-bit counter (Box-Muller on the first two words;
// v_cos_f32 takes its argument in revolutions).
DEV float philox_normal(uint64_t seed, uint32_t c0, uint32_t c1, uint64_t c23) {
    uint32_t ctr[4] = {c0, c1, (uint32_t)c23, (uint32_t)(c23 >> 32)};
    philox4x32(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float u1 = ((float)(ctr[0] >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
    const float u2 = (float)(ctr[1] >> 8) * (1.0f / 16777216.0f);            // [0, 1)
    return __builtin_amdgcn_sqrtf(-2.0f * flog(u1)) * __builtin_amdgcn_cosf(u2);
}

}  // namespace vaeb
