// latent.hpp -- the latent block folded into the wide GEMM phases (training step, Z <= 32).
//
// The latent-width GEMMs of the step are reductions over H (mu|lv = h [W4|W5]) followed
// by per-element work on only B x Z values.  As its own launch (P23) that ran on 7
// workgroups (one per 16 batch rows) for ~12 us.  Here:
//
//  enc_latent_kernel  (P1 + heads + sample): every 16x16 tile of h = tanh(X W3 + b3)
//      also multiplies its h tile by the matching 16 rows of [W4|W5] and publishes that
//      partial [mu|lv] slab; the LAST tile of each 16-row block to arrive sums the
//      block's slabs in fixed order (bitwise reproducible) and runs the element-wise
//      middle: eps, z = mu + exp(lv/2) eps, KL / LA terms (VAEB.py:41-47, 248-249,
//      322-325, 343).
//  decout_z_kernel    (dechid + decout): each K-slice wave recomputes its hd chunks
//      hd = tanh(z W1 + b1) as (W1^T z^T) -- whose MFMA output layout IS the A-operand
//      layout of the decoder GEMM -- so hd never makes a round trip through memory
//      before it is used; column tile 0 stores hd for the backward phases (VAEB.py:254).
//
// Slab hand-off (MI355X_MICROARCH.md visibility rules): slabs are stored write-through
// (sc1) with 16-byte stores, the storing wave drains (s_waitcnt vmcnt(0)) before one
// relaxed agent-scope fetch_add on the row block's counter, and the reducer reads every
// slab with sc1 loads: no fences, no spinning, correct for any XCD placement.  The
// reducer resets its counter (zeroed at context creation).
//
// Measured alternative (not kept): summing the slabs in the prologue of every
// decout workgroup instead -- each of the 49 column tiles of a row block then reads the
// block's 80 KB of slabs, and at ~90 GB/s of L2->CU bandwidth per CU that cost more
// (15.7 us decoder launch) than the arrival round trip here.
#pragma once
#include <type_traits>
#include "fused.hpp"
#include "kernels_aux.hpp"   // wgrad_body: the deferred dW2 workers of enc_latent16_w2_kernel

namespace vaeb {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

DEV void st4_sc1(rsrc_t b, uint32_t off, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), b, off, 0, 16);
}
DEV f32x4 ld4_sc1(rsrc_t b, uint32_t off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(b, off, 0, 16));
}

// Wave 0's slab stores are drained, then one ticket per tile; returns (to every thread)
// whether this workgroup is the last of its row block.
//
// Ordering: this is the hand-off form that MI355X_MICROARCH.md ("Workgroup dispatch, XCD
// placement & inter-workgroup visibility", Consumer bullet, `sc1` loads in place of the
// acquire) lists as valid without release / acquire fences when all four of its
// conditions hold, in the first row of its hand-off table:
//   (1) every load of the slab bytes is an sc1 load to registers (ld4_sc1, buffer form);
//   (2) the producer stores every slab byte sc1 (st4_sc1, 16 B);
//   (3) the only storing wave (wave 0) runs s_waitcnt vmcnt(0) after its stores and its
//       lane 0 then makes the ticket add, so the add follows the wait of every wave it
//       signals for;
//   (4) table row 1: one lane per storing workgroup adds to ONE unsharded agent-scope
//       counter, the workgroup whose add came last (told by the returned value) is the
//       consumer, its other waves load after the __syncthreads below; hipMalloc'd
//       memory, one workgroup per CU (224 / 256 tiles at MNIST-20).
// The relaxed add and the wavefront fence only keep the compiler from hoisting the slab
// loads above the ticket.  The fenced form (agent release before the add, agent acquire after
// it: the release writes back the XCD L2, the acquire invalidates the CU's L1) measured 2.9 us
// per step slower in round 2 (its A/B build was removed in round 6).
// NSW > 1: waves 0 .. NSW-1 stored slab bytes; each drains, the workgroup barrier follows,
// then lane 0 makes the one ticket add (the guide's producer form "every storing wave's
// s_waitcnt vmcnt(0), the workgroup's barrier, then ... flag/counter", the release replaced
// by the sc1 stores as above).
template <int NSW = 1>
DEV bool arrive_last(int* cnt, int target, int* sflag) {
    if constexpr (NSW > 1) {
        if ((int)threadIdx.x < 64 * NSW) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (threadIdx.x < 64) {
        if constexpr (NSW == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0) {
            const int old = __hip_atomic_fetch_add((gint*)cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *sflag = (old == target - 1);
        }
    }
    __syncthreads();
    const bool last = *sflag != 0;
    if (last && threadIdx.x == 0) __hip_atomic_store((gint*)cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the slab loads below the ticket
    return last;
}

// ---------------------------------------------------------------- atomic hand-off
// The alternative to slab + ticket + reducer: every contributing workgroup adds its
// partial of element e into ONE 64-bit accumulator with a returning agent-scope atomic,
// as a counted fixed-point number (two's complement)
//     inc = 2^59 + round(v * 2^32)      (count field: bits 59..63, fan-in <= 16)
// The add that brings the count field to n (the number of contributors) returns the complete
// sum, so that workgroup -- whichever it is -- finishes element e itself: no slab stores,
// no drain, no ticket, no reducer.  Every access to an accumulator is an atomic RMW on
// that one location (a single modification order), so no cross-location ordering, fence or
// cache rule is involved; the completer resets it (atomic store) for the next launch.
// Integer adds are associative: the sum, and so the result, is bitwise the same for any
// arrival order.
// Range guard: any subset of <= 16 partials with |v| < 2^17 sums below 2^53 in magnitude,
// so the fields above bit 53 always decode exactly.  A partial outside that range -- or NaN
// or inf (a diverging run) -- adds the count plus a POISON unit 2^54 (bits 54..58) instead
// of a value: the completer sees the poison and writes NaN, which then propagates through
// the step as it would on the slab path, and the accumulator is still reset cleanly.  The
// contributor also sets the sticky guard word (blk[kBlkFxErr] = acc_ml[-1], passed
// explicitly by BOTH hand-offs: acc_dz[-1] is a padding word of acc_ml's range; read and
// cleared by the step's ELBO reduction, which reports it as VAEB_ERR_NUMERIC to the host).
typedef __attribute__((address_space(1))) unsigned long long gu64;
constexpr double kFxScale = 4294967296.0;   // 2^32
constexpr float kFxMax = 131072.f;          // 2^17
constexpr int kFxCntShift = 59, kFxPoisonShift = 54;
DEV uint64_t fx_inc(float v, uint64_t* guard) {
    if (__builtin_expect(!(__builtin_fabsf(v) < kFxMax), 0)) {
        __hip_atomic_fetch_or((gu64*)guard, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return (1ull << kFxCntShift) + (1ull << kFxPoisonShift);
    }
    const int64_t q = (int64_t)__builtin_rint((double)v * kFxScale);
    return (1ull << kFxCntShift) + (uint64_t)q;
}
// adds inc to *p and returns the accumulator's new value (issue every add of a lane
// before decoding any: each decode waits for its add's return)
DEV uint64_t fx_add(uint64_t* p, uint64_t inc) {
    return __hip_atomic_fetch_add((gu64*)p, (unsigned long long)inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
           inc;
}
// true (and the element's sum in `out`: NaN when a contributor was poisoned) when tot is
// the value after the n-th add
DEV bool fx_done(uint64_t tot, int n, float& out) {
    const uint64_t hi = (tot + (1ull << (kFxPoisonShift - 1))) >> kFxPoisonShift;   // count * 32 + poison
    const float v = (float)((double)(int64_t)(tot - (hi << kFxPoisonShift)) * (1.0 / kFxScale));
    out = (hi & 31) ? __builtin_nanf("") : v;
    return (hi >> (kFxCntShift - kFxPoisonShift)) == (uint64_t)n;
}
DEV void fx_reset(uint64_t* p) { __hip_atomic_store((gu64*)p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// Accumulator e lives at word e * kFxStride: the atomics execute at the memory side, and
// consecutive 8-B words would put a whole hand-off (a few thousand accumulators, 32 adds
// each) on a handful of memory channels.
constexpr int kFxStride = 33;
constexpr int kFxMaxFanIn = 16;
DEV uint64_t* fx_at(uint64_t* base, int64_t e) { return base + e * kFxStride; }


// A tile's 16 rows x 2Z partials (Z <= 32) are handed off by all 512 threads of its
// workgroup, repacked through LDS so that no lane adds for a padding column: thread t takes
// elements t and t + 512 (NS = 2 slots when Z > 16, then the first is always present), element
// e = (column e >> 4, row e & 15).  Only the second slot's add sits in a branch, so at most
// one wait separates the two adds (a branch around every add made hipcc wait for each).
template <int NS, int NTH = 512>
struct FxSlots {
    uint64_t t[NS];
    bool ok[NS];
    int col[NS], row[NS];
    DEV void add(uint64_t* acc, uint64_t* guard, int64_t row0, int ncol, const float (*pm)[17], int ne) {
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            const int e = (int)threadIdx.x + NTH * u;
            ok[u] = e < ne;
            col[u] = ok[u] ? e >> 4 : 0;
            row[u] = e & 15;
        }
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            const uint64_t inc = fx_inc(pm[col[u]][row[u]], guard);
            uint64_t* p = fx_at(acc, (row0 + row[u]) * ncol + col[u]);
            t[u] = 0;
            if (NS == 2 && u == 0) t[u] = fx_add(p, inc);   // always present when NS == 2
            else if (ok[u]) t[u] = fx_add(p, inc);
        }
    }
};

// ----------------------------------------------------------------------------- P1'
// Grid (Mbp/16, ceil(H/16)), 512 threads: 8 waves split K = D.  Tile (bx, by) stores its
// partial [mu | lv] slab column-major: slab[((bx * nctH + by) * 2Z + c) * 16 + m]
// (c < Z: mu column c, c >= Z: lv column c - Z).
// Literal-FV steps append a.fv_rows grid rows of blocks that run fv_kernel's update over
// (mu, sigma) (kernels_aux.hpp: FvElem, same 16-byte group scheme), one thetaPrior partial
// per block: the update needs none of the step's data, so it fills the CUs the 16x16
// tiles leave idle instead of taking a launch of its own.
DEV void fv_stream_block(const FvFold& a, int fb, int nfb, double* sh) {
    const FvElem f{a.lr, a.eps, 1};
    const int64_t P = a.P, T = (int64_t)nfb * 512, n4 = P >> 2;
    const rsrc_t bm = mkbuf(a.mu, P * 4), bs = mkbuf(a.sg, P * 4);
    const rsrc_t bam = mkbuf(a.am, P * 4), bas = mkbuf(a.as, P * 4);
    double tp = 0;
    constexpr int U = 2;
    for (int64_t g0 = (int64_t)fb * 512 + threadIdx.x; g0 < n4; g0 += U * T) {
        uint32_t off[U];
        f32x4 m[U], s[U], a1[U], a2[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            fv_group(g0 + u * T, n4, off[u]);
            m[u] = bld4(bm, off[u]);
            s[u] = bld4(bs, off[u]);
            a1[u] = bld4(bam, off[u]);
            a2[u] = bld4(bas, off[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (off[u] == kOOB) continue;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float mm = m[u][k], ss = s[u][k], x1 = a1[u][k], x2 = a2[u][k];
                f(mm, ss, x1, x2, tp);
                m[u][k] = mm; s[u][k] = ss; a1[u][k] = x1; a2[u][k] = x2;
            }
            bst4(bam, off[u], a1[u]);
            bst4(bas, off[u], a2[u]);
            bst4(bm, off[u], m[u]);
            bst4(bs, off[u], s[u]);
        }
    }
    if (fb == 0 && threadIdx.x < (P & 3)) {
        const int64_t i = n4 * 4 + threadIdx.x;
        float m = a.mu[i], s = a.sg[i], x1 = a.am[i], x2 = a.as[i];
        f(m, s, x1, x2, tp);
        a.mu[i] = m; a.sg[i] = s; a.am[i] = x1; a.as[i] = x2;
    }
    tp = wave_sum64(tp);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = tp;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = sh[0];
#pragma unroll
        for (int w = 1; w < 8; ++w) r += sh[w];
        a.part[fb] = (float)r;
    }
}

// AT (atomic hand-off): tile (bx, by) adds its partial [mu | lv] into acc_ml; the add that
// completes an element stores mu or lv (+ bias).  Meanwhile waves 1-7 of column tile 0
// write the row block's eps (Philox keyed by the global row, the host buffer, or 0); z and
// the KL / LA terms are formed by decout_z_kernel<.., AT>.
// The encoder over CT 16-column h tiles per workgroup (wave_mainloop's NB = CT B operands).
struct PEncCT : PEnc {
    DEV f32x4 b4(int n, int k, int w) const { return mc4(bw, a.H, n + 16 * w, k, a.H, a.D); }
};

// CT: h column tiles per workgroup (1, or 2: half the contributors per latent element).
// NWV: waves splitting K (8; or 16 -- 1024-thread workgroups -- on the slab-only path HO = 3
// and the atomic hand-off HO = 1; the ticketed reducer HO = 0 keeps its 512-thread layout).
// red_ext (EXTRED): the K-slice reduction buffer (64 NWV CT f32x4) from the caller -- the
// deferred-dW2 encoder carves it from the LDS its dW2 workers use (enc_latent16_w2_kernel).
template <int NCT, int GCH, bool FV, int HO, int CT = 1, int NWV = 8, bool EXTRED = false>
DEV void enc_latent_body(const StepArgs& a, const FvFold& fvf, f32x4* red_ext = nullptr) {
    static_assert(NWV == 8 || (HO != 0 && !FV), "16 waves: no ticketed reducer, no FV stream");
    constexpr bool AT = HO == 1;
    constexpr int NTH = 64 * NWV;
    constexpr int NS = NWV == 16 ? 1 : NCT;   // atomic-add slots per thread: 32 Z <= 1024
    f32x4* red;
    if constexpr (EXTRED) {
        red = red_ext;
    } else {
        __shared__ f32x4 red_own[64 * NWV * CT];
        red = red_own;
    }
    __shared__ float hs[16][16 * CT + 4];
    __shared__ int sflag;
    __shared__ float pm[HO == 1 ? 64 : 1][17];   // the tile's [mu | lv] partials, [column][row]
    // contributors per row block: the grid's column workgroups (FV: rows beyond run the stream)
    // (grid extents from the arguments, not gridDim: reading the implicit arguments put one
    // more dependent scalar round trip ahead of every workgroup's first operand load)
    const int nctH = (a.H + 16 * CT - 1) / (16 * CT);
    const int gxE = a.Mbp >> 4;   // grid: (Mbp / 16, nctH (+ FV stream rows))
    if (FV && (int)blockIdx.y >= nctH) {
        fv_stream_block(fvf, (blockIdx.y - nctH) * gxE + blockIdx.x, fvf.rows * gxE, reinterpret_cast<double*>(red));
        return;
    }
    VAEB_STAMP(a, 0);
    PEncCT p{PEnc{a, nullptr, a.Mbp, a.H, a.D}};
    p.prepare();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, q = lane >> 4;
    const int lin = xcd_remap(blockIdx.x + blockIdx.y * gxE, gxE * nctH);
    const int bx = lin % gxE, by = lin / gxE;
    const int m0 = bx * 16, n0 = by * 16 * CT;
    const int Z = a.Z, H = a.H;
    const rsrc_t bs = mkbuf(a.slab_ml, (int64_t)gxE * nctH * 2 * Z * 16 * 4);

    // Row-parallel epilogue: phase A -- wave w < 4 CT finishes row group r = w & 3 of h column
    // tile c = w >> 2 (sum of the 8 K-slice partials, bias, tanh, h); phase B -- wave w < 2 NCT
    // forms part w of the tile's [mu | lv] partial (mu / lv of latent tile w >> 1) from all of
    // h through LDS.  (One wave running both phases serially was ~2.5 us of the launch.)  The
    // ticketed slab form (HO 0) keeps its single storing wave for phase B (arrive_last).
    constexpr bool kOneB = HO == 0;
    const int ca = wave >> 2, ra = wave & 3;
    const bool wa = wave < 4 * CT, wb = kOneB ? wave == 0 : wave < 2 * NCT;
    PEnc::Pre pre{};
    f32x4 bw[CT][kOneB ? 2 * NCT : 1];
    if (wa) pre = p.prefetch(m0, n0 + 16 * ca);
    if (wb) {
        const rsrc_t bw4 = mkbuf(a.W4, (int64_t)H * Z * 4), bw5 = mkbuf(a.W5, (int64_t)H * Z * 4);
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int u = 0; u < (kOneB ? 2 * NCT : 1); ++u) {
                const int w = kOneB ? u : wave;
                bw[c][u] = mc4((w & 1) ? bw5 : bw4, Z, (w >> 1) * 16 + li, n0 + 16 * c + 4 * q, Z, H);
            }
    }
    // AT: the bias of each element this thread may complete (column c: b4[c] | b5[c - Z])
    float bias[NS];
    if constexpr (AT) {
        const rsrc_t b4 = mkbuf(a.b4, (int64_t)Z * 4), b5 = mkbuf(a.b5, (int64_t)Z * 4);
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            const int e = (int)threadIdx.x + NTH * u, c = e >> 4;
            const bool ok = e < 32 * Z;
            bias[u] = bld(b4, ok && c < Z ? (uint32_t)c * 4u : kOOB) + bld(b5, ok && c >= Z ? (uint32_t)(c - Z) * 4u : kOOB);
        }
    }
    f32x4 acc[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[c] = zero4();
    wave_mainloop<CT, NWV, GCH>(p, m0 + li, n0 + li, p.K, wave, acc);
    VAEB_STAMP(a, 1);
    float* redh = reinterpret_cast<float*>(red);   // [c][r][slice][lane]: CT * 2048 floats
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) redh[((c * 4 + r) * NWV + wave) * 64 + lane] = acc[c][r];
    __syncthreads();
    if (a.order && bx == 0 && by == 0 && threadIdx.x == 0) *a.cur_batch = a.cursor[kCtlNext];
    if (wa) {
        float t = redh[((ca * 4 + ra) * NWV) * 64 + lane];
#pragma unroll
        for (int sl = 1; sl < NWV; ++sl) t += redh[((ca * 4 + ra) * NWV + sl) * 64 + lane];
        const int n = n0 + 16 * ca + li, m = m0 + 4 * q + ra;
        const float hv = (m < a.Mb && n < H) ? ftanh(t + pre.b) : 0.f;
        if (n < H) a.h[(int64_t)m * H + n] = hv;
        hs[4 * q + ra][16 * ca + li] = hv;
    }
    __syncthreads();
    if (wb) {
        // partial [mu|lv] of this tile: (16 x 16 CT h) . (16 CT rows of [W4|W5])
        f32x4 av[CT];
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int s = 0; s < 4; ++s) av[c][s] = hs[li][16 * c + 4 * q + s];
        const int64_t base = ((int64_t)bx * nctH + by) * 2 * Z;
        auto part = [&](int u) {
            f32x4 v = mfma4(av[0], bw[0][u], zero4());
#pragma unroll
            for (int c = 1; c < CT; ++c) v = mfma4(av[c], bw[c][u], v);
            return v;
        };
#pragma unroll
        for (int u = 0; u < (kOneB ? 2 * NCT : 1); ++u) {
            const int w = kOneB ? u : wave;
            const f32x4 sv = part(u);
            const int nz = (w >> 1) * 16 + li;   // latent column of this lane
            if constexpr (HO == 1) {
                if (nz < Z)
#pragma unroll
                    for (int r = 0; r < 4; ++r) pm[(w & 1) * Z + nz][4 * q + r] = sv[r];
            } else if constexpr (HO == 3) {
                // the decoder launch sums the slabs (decout_z_kernel<.., ZM = 2>): plain stores,
                // made visible by the kernel boundary
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, sv), bs,
                                                       nz < Z ? (uint32_t)(((base + (w & 1) * Z + nz) * 16 + 4 * q) * 4) : kOOB, 0, 0);
            } else {
                st4_sc1(bs, nz < Z ? (uint32_t)(((base + (w & 1) * Z + nz) * 16 + 4 * q) * 4) : kOOB, sv);
            }
        }
    }
    if constexpr (HO == 3) {
        VAEB_STAMP(a, 2);
        return;
    }
    if constexpr (AT) {
        __syncthreads();
        FxSlots<NS, NTH> fx;
        fx.add(a.acc_ml, a.acc_ml - 1, m0, 2 * Z, pm, 32 * Z);
        if (by == 0) {   // the row block's eps, while the adds are in flight
            // the row base comes from `next` (kCtlNext): cur_batch is written by tile (0,0)
            // of this same launch, which need not have run yet
            const int64_t grow0 =
                (a.order ? (int64_t)ld_launch_const(a.cursor + kCtlNext) * a.row_base_mul : 0) + a.row_base_add;
            const uint64_t c23 = philox_c23(a.step ? *a.step : 0, a.domain);
            const int per = 16 * Z;
            for (int id = threadIdx.x; id < a.L * per; id += NTH) {
                const int l = id / per, ml = (id - l * per) / Z, j = id - l * per - ml * Z;
                const int m = m0 + ml;
                float e = 0.f;
                if (m < a.Mb) {
                    if (a.eps_mode == 0) e = philox_normal(a.seed, (uint32_t)(grow0 + m), (uint32_t)(l * Z + j), c23);
                    else if (a.eps_mode == 1) e = a.eps_in[((int64_t)l * a.eps_in_ld + m) * Z + j];
                }
                a.eps[((int64_t)l * a.Mbp + m) * Z + j] = e;
            }
        }
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            float v;
            if (fx.ok[u] && fx_done(fx.t[u], nctH, v)) {
                const int c = fx.col[u], m = m0 + fx.row[u];
                float* dst = c < Z ? a.mu : a.lv;
                dst[(int64_t)m * Z + (c < Z ? c : c - Z)] = m < a.Mb ? v + bias[u] : 0.f;
                fx_reset(fx_at(a.acc_ml, (int64_t)m * 2 * Z + c));
            }
        }
        VAEB_STAMP(a, 2);
        return;
    }
    VAEB_STAMP(a, 2);
    if (!arrive_last(a.cnt_ml + bx, nctH, &sflag)) return;
    VAEB_STAMP(a, 3);

    // ---- reducer (the last tile of row block bx): the element-wise operands ride the
    // same round trip as the slab loads
    const int ml = threadIdx.x >> 5, n = threadIdx.x & 31;
    const int m = m0 + ml;
    const bool valid = n < Z && m < a.Mb;
    const float b4n = bld(mkbuf(a.b4, (int64_t)Z * 4), n < Z ? (uint32_t)n * 4u : kOOB);
    const float b5n = bld(mkbuf(a.b5, (int64_t)Z * 4), n < Z ? (uint32_t)n * 4u : kOOB);
    float epre[kLP];
    {
        const rsrc_t be = mkbuf(a.eps_in, a.eps_mode == 1 ? (int64_t)a.L * a.eps_in_ld * Z * 4 : 0);
#pragma unroll
        for (int l = 0; l < kLP; ++l)
            epre[l] = bld(be, (a.eps_mode == 1 && l < a.L && valid) ? (uint32_t)((l * a.eps_in_ld + m) * Z + n) * 4u : kOOB);
    }
    // the row base comes from `next` (kCtlNext): cur_batch is written by tile (0,0) of
    // this same launch, which need not have run yet
    const int64_t grow0 = (a.order ? (int64_t)ld_launch_const(a.cursor + kCtlNext) * a.row_base_mul : 0) + a.row_base_add;
    const int64_t stp = a.step ? *a.step : 0;
    float mu = 0.f, lv = 0.f;
    const int NF4 = 8 * Z;                  // float4 per slab (2Z columns x 16 rows)
    const int NP = 512 / NF4;               // slab partitions (threads >= NP * NF4 idle)
    if constexpr (HO == 0) {
        const int f = threadIdx.x % NF4, part = threadIdx.x / NF4;
        const int64_t first = (int64_t)bx * nctH * NF4;
        constexpr int SV = 12;
        f32x4 sum = zero4();
        for (int c0 = part; c0 < nctH; c0 += SV * NP) {
            f32x4 v[SV];
#pragma unroll
            for (int u = 0; u < SV; ++u) {
                const int ct = c0 + u * NP;
                v[u] = ld4_sc1(bs, (part < NP && ct < nctH) ? (uint32_t)((first + (int64_t)ct * NF4 + f) * 16) : kOOB);
            }
#pragma unroll
            for (int u = 0; u < SV; ++u) sum += v[u];
        }
        red[threadIdx.x] = sum;
        __syncthreads();
        VAEB_STAMP(a, 4);
        auto at = [&](int c) {  // element (column c, row ml) of the summed slab
            const int ff = (c * 16 + ml) >> 2, comp = ml & 3;
            float v = 0.f;
            for (int pp = 0; pp < NP; ++pp) v += red[pp * NF4 + ff][comp];
            return v;
        };
        if (n < Z) { mu = at(n); lv = at(Z + n); }
    }
    mu = valid ? mu + b4n : 0.f;
    lv = valid ? lv + b5n : 0.f;
    const float sd = fexp(0.5f * lv);
    const float elv = fexp(lv);
    const uint64_t c23 = philox_c23(stp, a.domain);
    for (int l = 0; l < a.L; ++l) {
        float e = 0.f;
        if (valid) {
            if (a.eps_mode == 0) e = philox_normal(a.seed, (uint32_t)(grow0 + m), (uint32_t)(l * Z + n), c23);
            else if (a.eps_mode == 1) e = (l < kLP) ? epre[l] : a.eps_in[((int64_t)l * a.eps_in_ld + m) * Z + n];
        }
        const float z = valid ? mu + sd * e : 0.f;
        if (n < Z) {
            const int64_t o = ((int64_t)l * a.Mbp + m) * Z + n;
            a.eps[o] = e;
            a.z[o] = z;
        }
        if (a.est == EST_LA) {
            const float d = z - mu;
            float f = valid ? (-0.5f * z * z) - (-0.5f * lv - 0.5f * d * d / elv) : 0.f;
            f = sum32(f);
            if (n < a.nctZ) a.la_part[((int64_t)l * a.Mbp + m) * a.nctZ + n] = (n == 0) ? f : 0.f;
        }
    }
    if (n < Z) {
        a.mu[(int64_t)m * Z + n] = mu;
        a.lv[(int64_t)m * Z + n] = lv;
    }
    if (a.est != EST_LA) {
        float kl = valid ? 0.5f * (1.f + lv - mu * mu - elv) : 0.f;
        kl = sum32(kl);
        if (n < a.nctZ) a.kl_part[(int64_t)m * a.nctZ + n] = (n == 0) ? kl : 0.f;
    }
    VAEB_STAMP(a, 5);
}
template <int NCT, int GCH, int HO, int CT>
__global__ __launch_bounds__(512) void enc_latent_kernel(StepArgs a) {
    enc_latent_body<NCT, GCH, false, HO, CT>(a, FvFold{});
}
template <int NCT, int GCH, int HO, int CT>
__global__ __launch_bounds__(512) void enc_latent_fv_kernel(StepArgs a, FvFold f) {
    enc_latent_body<NCT, GCH, true, HO, CT>(a, f);
}
// the slab-only (HO = 3, CT = 2) and atomic hand-off (HO = 1) encoders on 16 waves
template <int NCT, int GCH, int HO, int CT>
__global__ __launch_bounds__(1024) void enc_latent16_kernel(StepArgs a) {
    enc_latent_body<NCT, GCH, false, HO, CT, 16>(a, FvFold{});
}

// The same encoder with the PREVIOUS step's dW2 (| dW6) tiles + Adagrad on the CUs it leaves
// idle (the deferred dW2, vaeb_hip.hip vaeb_ctx::dw2_defer): the encoder's 112 workgroups
// take 112 of 256 CUs at MNIST, and W2 is first read again by this step's decoder launch.
// Grid rows >= rows_enc are dW2 workers, two 64 x (16 TS) tiles each (waves 0-7 and 8-15,
// wgrad_body's 512-thread tile on its own half of the LDS); they read hd / dA2 of the previous
// step (intact until this step's decoder launch) and theta from the other arena, and write
// W2' into the arena this step reads (which the encoder does not touch).  *pend == 0
// (nothing pending: the first step, or a flush since) drops their stores.  LDS: two tiles' (sa,
// sb) = 139 KB, the encoder's K-slice reduction buffer (32 KB) carved from the same block.
template <int NCT, int GCH, int HO, int CT, bool VEC, int TS>
__global__ __launch_bounds__(1024) void enc_latent16_w2_kernel(StepArgs a, WGradArgs w, const int* pend, int rows_enc) {
    __shared__ __attribute__((aligned(16))) float lds[4 * kWKB * kWP];
    static_assert(sizeof(float) * 4 * kWKB * kWP >= sizeof(f32x4) * 64 * 16 * CT, "LDS union");
    if ((int)blockIdx.y >= rows_enc) {
        const int half = (int)threadIdx.x >> 9;
        const int bid = 2 * (((int)blockIdx.y - rows_enc) * (a.Mbp >> 4) + (int)blockIdx.x) + half;
        float (*sa)[kWP] = reinterpret_cast<float(*)[kWP]>(lds + half * 2 * kWKB * kWP);
        wgrad_body<VEC, 8, TS>(w, w.g[0], bid, sa, sa + kWKB, pend);
        return;
    }
    enc_latent_body<NCT, GCH, false, HO, CT, 16, true>(a, FvFold{}, reinterpret_cast<f32x4*>(lds));
}

// ----------------------------------------------------------------------------- P4'
// Grid (Me/16, ceil(D/16)), 512 threads.  Wave w owns the 64-wide K blocks
// kb = 64 (w + 8 g); within a block, sub-chunk u (0..3) of the hd^T product puts hd
// column kb + 4 i + u on output row i, so one float4 of W1 feeds all four sub-chunks
// and lane (m, q) ends with hd[m][kb + 16 q + 4 r + u] -- the decoder GEMM's A operand
// at MFMA step r, matched by W2 row kb + 16 q + 4 r + u on the B side.
// ZS = ceil(Z / 4): the hd^T product runs ZS MFMA k-steps (latent 4t + q at step t).
// V1 (host-chosen: H % 4 == 0, W1 / b1 16-byte aligned) selects the 16-byte W1 / b1
// loads at compile time: with a runtime choice the loads sat in branches and hipcc drained
// vmcnt at each, serialising the z, W1 / b1 and W2 round trips.  The x rows for the
// likelihood are resolved (scalar load of cur_batch) only after wave 0 has issued its
// first block's operand loads.
// AT (atomic hand-off, enc_latent_body<.., AT>): z = mu + exp(lv / 2) eps is formed here
// from mu, lv and eps (all written by the encoder launch), and column tile 0 stores z and
// the row's KL (LB / FV, plane 0) or LA partial for the backward and the ELBO.
// ZM: 0 = z read from memory; 1 = AT (z formed from mu, lv, eps that the encoder launch
// wrote); 2 = the encoder's CT = 2 partial [mu | lv] slabs (enc_latent_body<.., HO = 3, 2>,
// ceil(H / 32) per row block) summed here in fixed order, + bias, eps drawn here, and column
// tile 0 stores mu, lv, eps, z and the KL / LA terms for the backward and the ELBO.
// CT: 16-column output tiles per workgroup (1, or 2 for the Bernoulli decoder: one workgroup
// per CU at MNIST instead of 343 workgroups on 256 CUs, and the W1 / slab reads and the hd
// recompute shared by both tiles).  NT = NB * CT accumulators, tile-major.
template <int NB, int ZS, bool V1, int ZM, int CT>
DEV void decout_z_body(const StepArgs& a) {
    constexpr bool AT = ZM != 0;
    constexpr int CW = 16 * CT;   // output columns per workgroup
    constexpr int NT = NB * CT;
    using PD = PDecOut;
    VAEB_STAMP(a, 0);
    PD p{a, nullptr, a.Me, a.D, a.H};
    p.prepare_at(nullptr);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, q = lane >> 4;
    const int gx = a.Me >> 4, gy = (a.D + CW - 1) / CW;   // the grid (no implicit-argument load)
    const int lin = xcd_remap(blockIdx.x + blockIdx.y * gx, gx * gy);
    // CT = 2 (the Bernoulli two-tile decoder): consecutive logical ids (one XCD's run under
    // xcd_remap) share a row block, so each XCD's L2 fetches the encoder slabs and x rows of ~1 row
    // block instead of all 7 (the W2 column panels then spread over the XCDs): round 5, alternating
    // 2000-step runs, MNIST 34.30 / 34.32 / 34.34 us against 34.46 / 34.46 column-major
    // (-DVAEB_DEC_COLMAJOR).  CT = 1 (Gaussian, Frey) keeps the column-major order: 30.15 / 30.23
    // row-major against 29.77 / 29.83 us.
    constexpr bool kRowMajor = CT == 2;
    const int bxr = kRowMajor ? lin / gy : lin % gx, byr = kRowMajor ? lin % gy : lin / gx;
    const int m0 = bxr * 16, n0 = byr * CW;
    const int Z = a.Z, H = a.H;
    const bool col0 = byr == 0;
    const bool rowok = ((m0 + li) % a.Mbp) < a.Mb;
    const rsrc_t bw1 = mkbuf(a.W1, (int64_t)Z * H * 4);
    const rsrc_t bb1 = mkbuf(a.b1, (int64_t)H * 4);
    constexpr bool v1 = V1;
    typename PD::PreRow pre{};
    f32x4 acc[NT];
#pragma unroll
    for (int w = 0; w < NT; ++w) acc[w] = zero4();
    // W1^T rows kb + 4 li + (0..3) at latent 4t + q; b1 at kb + 16 q + 4 r + (0..3); W2 rows
    // kb + 16 q + 4 r + u.  The first block's loads are issued BEFORE the z prologue (whose
    // own loads -- z, mu / lv / eps, or the encoder's slabs -- they do not depend on), so
    // both round trips overlap (MNIST ZM 0 decout 10.5 -> 10.2 us); a block past H reads
    // zeros.  ZM 2 spreads its slab sum over all 512 threads (at most kSlabPer loads each)
    // so that the hoisted block still fits 128 VGPRs (round 2's 16 slab float4s per thread
    // beside it spilled).
    f32x4 w1v[ZS], b1v[4];
    float w2b[4][4][NT];
    auto load_block = [&](int kb) {
#pragma unroll
        for (int t = 0; t < ZS; ++t) {
            const int c = 4 * t + q, k = kb + 4 * li;
            w1v[t] = kc4(bw1, H, c, k, Z, H, v1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) b1v[r] = kc4(bb1, 0, 0, kb + 16 * q + 4 * r, 1, H, v1);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int w = 0; w < NT; ++w) {
                    const int k = kb + 16 * q + 4 * r + u;
                    w2b[u][r][w] = p.b1(n0 + 16 * (w / NB) + li, k, w % NB);
                }
    };
    // ZM 2: the first kSlabPer slab loads of each thread are issued BEFORE the weight block:
    // vmcnt counts in issue order, so the slab sum (the critical path to z) then waits only for
    // its own loads, not for the 25 weight-block loads behind them.
    constexpr int kSlabPer = 6;
    f32x4 sv0[ZM == 2 ? kSlabPer : 1];
    const int nctS = (H + 31) >> 5, nf4S = 8 * Z;
    const int npS = 512 / nf4S;   // nf4 <= 256 (Z <= 32): np >= 2
    const int fS = (int)threadIdx.x % nf4S, partS = (int)threadIdx.x / nf4S;
    const rsrc_t bsl = mkbuf(a.slab_ml, ZM == 2 ? (int64_t)(a.Mbp >> 4) * nctS * nf4S * 16 : 0);
    const int64_t firstS = (int64_t)((m0 % a.Mbp) >> 4) * nctS * nf4S + fS;
    if constexpr (ZM == 2) {
#pragma unroll
        for (int u = 0; u < kSlabPer; ++u) {
            const int ct = partS + u * npS;
            sv0[u] = bld4(bsl, (partS < npS && ct < nctS) ? (uint32_t)((firstS + (int64_t)ct * nf4S) * 16) : kOOB);
        }
    }
    load_block(64 * wave);
    float zb[ZS];
    if constexpr (!AT) {
        const rsrc_t bz = mkbuf(a.z, (int64_t)a.Me * Z * 4);
#pragma unroll
        for (int t = 0; t < ZS; ++t) zb[t] = bld(bz, (4 * t + q < Z) ? (uint32_t)((m0 + li) * Z + 4 * t + q) * 4u : kOOB);
    } else {
        // the row block's 16 x Z block of z, once per workgroup: thread (ml, j) loads mu, lv
        // and eps of one element (coalesced), the waves then read their fragments from LDS
        __shared__ float zs[16][33];
        __shared__ float gs[16][33];
        __shared__ float msum[ZM >= 2 ? 64 : 1][17];   // ZM 2: summed [mu | lv], [column][row]
        __shared__ f32x4 spart[ZM == 2 ? 512 : 1];      // ZM 2: per-partition slab sums
        const int per = 16 * Z;
        const int l = m0 / a.Mbp;                 // a 16-row block never straddles two planes
        const int i0 = m0 - l * a.Mbp;
        // ZM 2: the element phase's own operands (b4 / b5 of its latent column, the step
        // counter, the host eps) are loaded BEFORE the slab round trip, so the element phase
        // after the barrier starts from registers (they were dependent loads behind it)
        float b4p = 0.f, b5p = 0.f, epre = 0.f;
        int64_t stp = 0, grow0p = 0;
        if constexpr (ZM >= 2) {
            if ((int)threadIdx.x < per) {
                const int ml = threadIdx.x / Z, j = threadIdx.x - ml * Z;
                b4p = a.b4[j];
                b5p = a.b5[j];
                if (a.eps_mode == 1 && i0 + ml < a.Mb) epre = a.eps_in[((int64_t)l * a.eps_in_ld + i0 + ml) * Z + j];
            }
            stp = a.step ? *a.step : 0;
            grow0p = (a.order ? (int64_t)ld_launch_const(a.cursor + kCtlNext) * a.row_base_mul : 0) + a.row_base_add;
        }
        if constexpr (ZM == 2) {
            // float4 f (column f >> 2, rows 4 (f & 3) .. + 3) of the row block's nct slabs:
            // partition part = t / nf4 of the 512 threads sums slabs part, part + np, ... in
            // order (at most kSlabPer loads in flight per thread), then thread f adds the np
            // partition sums in order -- a fixed order, so the result is deterministic
            const int nct = nctS, nf4 = nf4S, np = npS, f = fS, part = partS;
            const int64_t first = firstS;
            f32x4 sum = zero4();
#pragma unroll
            for (int u = 0; u < kSlabPer; ++u) sum += sv0[u];
            for (int c0 = part + kSlabPer * np; c0 < nct; c0 += kSlabPer * np) {
                f32x4 v[kSlabPer];
#pragma unroll
                for (int u = 0; u < kSlabPer; ++u) {
                    const int ct = c0 + u * np;
                    v[u] = bld4(bsl, (part < np && ct < nct) ? (uint32_t)((first + (int64_t)ct * nf4) * 16) : kOOB);
                }
#pragma unroll
                for (int u = 0; u < kSlabPer; ++u) sum += v[u];
            }
            spart[threadIdx.x] = sum;
            __syncthreads();
            if ((int)threadIdx.x < nf4) {
                f32x4 t = spart[threadIdx.x];
                for (int pp = 1; pp < np; ++pp) t += spart[pp * nf4 + threadIdx.x];
                const int c = threadIdx.x >> 2, mq = threadIdx.x & 3;
#pragma unroll
                for (int k = 0; k < 4; ++k) msum[c][4 * mq + k] = t[k];
            }
            __syncthreads();
            VAEB_STAMP(a, 6);   // (timeline build) slab sum done
        }
        if ((int)threadIdx.x < per) {
            const int ml = threadIdx.x / Z, j = threadIdx.x - ml * Z;
            const int i = i0 + ml;
            const bool rv = i < a.Mb;
            float mu, lv, e;
            if constexpr (ZM >= 2) {
                mu = rv ? msum[j][ml] + b4p : 0.f;
                lv = rv ? msum[Z + j][ml] + b5p : 0.f;
                // eps as the encoder's reducer draws it (Philox keyed by the global row)
                e = 0.f;
                if (rv) {
                    if (a.eps_mode == 0) e = philox_normal(a.seed, (uint32_t)(grow0p + i), (uint32_t)(l * Z + j), philox_c23(stp, a.domain));
                    else if (a.eps_mode == 1) e = epre;
                }
                if (col0) {
                    a.eps[((int64_t)l * a.Mbp + i) * Z + j] = e;
                    if (l == 0) {
                        a.mu[(int64_t)i * Z + j] = mu;
                        a.lv[(int64_t)i * Z + j] = lv;
                    }
                }
            } else {
                mu = a.mu[(int64_t)i * Z + j];
                lv = a.lv[(int64_t)i * Z + j];
                e = a.eps[((int64_t)l * a.Mbp + i) * Z + j];
            }
            const float z = rv ? mu + fexp(0.5f * lv) * e : 0.f;
            zs[ml][j] = z;
            if (col0) {
                a.z[((int64_t)l * a.Mbp + i) * Z + j] = z;
                const float elv = fexp(lv);
                float g;
                if (a.est == EST_LA) {
                    const float d = z - mu;
                    g = (-0.5f * z * z) - (-0.5f * lv - 0.5f * d * d / elv);
                } else {
                    g = 0.5f * (1.f + lv - mu * mu - elv);
                }
                gs[ml][j] = rv ? g : 0.f;
            }
        }
        __syncthreads();
        VAEB_STAMP(a, 7);   // (timeline build) z formed
#pragma unroll
        for (int t = 0; t < ZS; ++t) zb[t] = (4 * t + q < Z) ? zs[li][4 * t + q] : 0.f;
        if (col0 && threadIdx.x < 16 && (a.est == EST_LA || l == 0)) {
            float f = 0.f;
            for (int j = 0; j < Z; ++j) f += gs[threadIdx.x][j];
            const int i = i0 + threadIdx.x;
            float* dst = a.est == EST_LA ? a.la_part + ((int64_t)l * a.Mbp + i) * a.nctZ : a.kl_part + (int64_t)i * a.nctZ;
            for (int n = 0; n < a.nctZ; ++n) dst[n] = n == 0 ? f : 0.f;
        }
    }
    for (int kb = 64 * wave; kb < H; kb += 64 * 8) {
        if (kb != 64 * wave) load_block(kb);
        if (kb == 64 * wave && wave < 4 * CT) {   // epilogue waves, first block: its loads are in flight
            p.x = x_rows(a);
            pre = p.prefetch_row(m0, n0 + 16 * (wave >> 2), wave & 3);
        }
        f32x4 hv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            f32x4 t = zero4();
#pragma unroll
            for (int st = 0; st < ZS; ++st) t = __builtin_amdgcn_mfma_f32_16x16x4f32(w1v[st][u], zb[st], t, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) hv[u][r] = rowok ? ftanh(t[r] + b1v[r][u]) : 0.f;
        }
        if (col0) {  // hd[m][kb + 16q + 4r + u] for u = 0..3: one float4 per r
            float* dst = a.hd + (int64_t)(m0 + li) * H;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = kb + 16 * q + 4 * r;
                const f32x4 o = {hv[0][r], hv[1][r], hv[2][r], hv[3][r]};
                if (v1) {
                    if (k < H) *reinterpret_cast<f32x4*>(dst + k) = o;
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (k + u < H) dst[k + u] = o[u];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int w = 0; w < NT; ++w)
                    acc[w] = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[u][r], w2b[u][r][w], acc[w], 0, 0, 0);
    }
    if (wave < 4 * CT && 64 * wave >= H) {   // an epilogue wave without a K block (H <= 192)
        p.x = x_rows(a);
        pre = p.prefetch_row(m0, n0 + 16 * (wave >> 2), wave & 3);
    }
    VAEB_STAMP(a, 1);
    // Row-parallel epilogue: the 8 K-slice partials go through LDS as [slice][tile][r][lane],
    // then wave r (< 4) sums row group r of the tile (slices in order 0..7) and finishes it.
    // One wave running all four row groups serially was ~0.55 us per group (a single wave's
    // dependent chain of likelihood, stores and the row sum): 2.2 us of the launch.
    // (CT = 2: wave w < 8 finishes row group w & 3 of tile w >> 2)
    __shared__ float redr[8][NT][4][64];
#pragma unroll
    for (int w = 0; w < NT; ++w)
#pragma unroll
        for (int r = 0; r < 4; ++r) redr[wave][w][r][lane] = acc[w][r];
    __syncthreads();
    VAEB_STAMP(a, 2);
    const int et = wave >> 2, er = wave & 3;
    if (wave >= 4 * CT || n0 + 16 * et >= a.D) return;
    float c[NB];
#pragma unroll
    for (int w = 0; w < NB; ++w) {
        float t = redr[0][et * NB + w][er][lane];
#pragma unroll
        for (int s = 1; s < 8; ++s) t += redr[s][et * NB + w][er][lane];
        c[w] = t;
    }
    VAEB_STAMP_SYNC(a, 4);   // (timeline build) the epilogue's operands landed
    p.epilogue_row(m0, n0 + 16 * et, er, c[0], c[NB - 1], pre);
    VAEB_STAMP(a, 3);
    VAEB_STAMP_SYNC(a, 5);   // (timeline build) the epilogue's stores drained
}
template <int NB, int ZS, bool V1, int ZM>
__global__ __launch_bounds__(512, 4) void decout_z_kernel(StepArgs a) {
    decout_z_body<NB, ZS, V1, ZM, 1>(a);
}
// two 16-column tiles per workgroup (Bernoulli): one workgroup per CU, so the full register file
template <int ZS, bool V1, int ZM>
__global__ __launch_bounds__(512, 2) void decout_z2_kernel(StepArgs a) {
    decout_z_body<1, ZS, V1, ZM, 2>(a);
}

}  // namespace vaeb
