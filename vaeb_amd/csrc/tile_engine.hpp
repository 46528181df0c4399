// tile_engine.hpp -- fp32 MFMA tile engine for gfx950 (CDNA4).
//
// Every contraction of the SGVB step (VAEB.py:245-265 forward, the T.grad backward of
// VAEB.py:397) is C[M x N] = A[M x K] * B[K x N] with small, awkward shapes (M = batch
// rows = 100, K as small as Z = 20, N as small as Z).  One wave owns a 16x16 output tile
// and runs v_mfma_f32_16x16x4_f32 (exact f32, 64 FLOP/clk/SIMD = the f32 peak of the
// chip) over its share of K; a 256-thread workgroup holds WM x WN tiles x KS K-slices
// (WM*WN*KS == 4 waves), and K-slices are summed through LDS before the fused epilogue.
//
// Operand feeding (per lane l, i = l & 15, q = l >> 4, chunk c of 16 k-values):
//   the MFMA's k-group q is fed k = 16c + 4q + s at step s = 0..3, so each lane needs
//   FOUR CONSECUTIVE k at its fixed row (A) / column (B): one 16-byte load when the
//   operand is K-contiguous, four coalesced scalar loads when it is M/N-contiguous.
// C/D mapping of 16x16x4 f32: col = l & 15, row = 4*(l >> 4) + r  (r = 0..3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace vaeb {

DEV f32x4 zero4() { f32x4 z = {0.f, 0.f, 0.f, 0.f}; return z; }

// K-contiguous operand: element (r, k) = p[r * ld + k]; rows >= rlim or k >= klim read 0.
DEV f32x4 ld4_kc(const float* __restrict__ p, int ld, int r, int k, int rlim, int klim, bool vec) {
    f32x4 v = zero4();
    if (r < rlim) {
        const float* q = p + (int64_t)r * ld + k;
        if (vec && k + 3 < klim && ((reinterpret_cast<uintptr_t>(q) & 15) == 0)) {
            v = *reinterpret_cast<const f32x4*>(q);
        } else {
            if (k + 0 < klim) v.x = q[0];
            if (k + 1 < klim) v.y = q[1];
            if (k + 2 < klim) v.z = q[2];
            if (k + 3 < klim) v.w = q[3];
        }
    }
    return v;
}

// M/N-contiguous operand: element (r, k) = p[k * ld + r].
DEV f32x4 ld4_mc(const float* __restrict__ p, int ld, int r, int k, int rlim, int klim) {
    f32x4 v = zero4();
    if (r < rlim) {
        const float* q = p + (int64_t)k * ld + r;
        if (k + 0 < klim) v.x = q[0];
        if (k + 1 < klim) v.y = q[(int64_t)ld];
        if (k + 2 < klim) v.z = q[(int64_t)2 * ld];
        if (k + 3 < klim) v.w = q[(int64_t)3 * ld];
    }
    return v;
}

DEV f32x4 mfma4(f32x4 a, f32x4 b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
    return c;
}

// Sum over the 16 lanes that share l >> 4 (one output row group of the C/D map).
DEV float sum16(float v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    return v;
}

// The wave-level main loop: accumulate NB tiles that share the A operand.
// P must provide:  f32x4 a4(int m, int k) const;  f32x4 b4(int n, int k, int which) const;
template <int NB, int KS, class P>
DEV void wave_mainloop(const P& p, int m, int n, int K, int kslice, f32x4 (&acc)[NB]) {
    const int lane = threadIdx.x & 63;
    const int kq = 4 * (lane >> 4);
    const int nch = (K + 15) >> 4;
    int c = kslice;
    // 4 chunks in flight per iteration (16 VGPR of A + 16*NB of B) to hide L2 latency.
    for (; c + 3 * KS < nch; c += 4 * KS) {
        f32x4 a[4], b[4][NB];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = (c + u * KS) * 16 + kq;
            a[u] = p.a4(m, k);
#pragma unroll
            for (int w = 0; w < NB; ++w) b[u][w] = p.b4(n, k, w);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int w = 0; w < NB; ++w) acc[w] = mfma4(a[u], b[u][w], acc[w]);
    }
    for (; c < nch; c += KS) {
        const int k = c * 16 + kq;
        f32x4 a = p.a4(m, k);
#pragma unroll
        for (int w = 0; w < NB; ++w) acc[w] = mfma4(a, p.b4(n, k, w), acc[w]);
    }
}

// Generic tile kernel.  Grid: x = M tiles / WM, y = N tiles / WN.  P also provides
//   int M, N, K;  void prepare();  void epilogue(int m0, int n0, const f32x4 (&acc)[NB]) const;
template <int WM, int WN, int KS, int NB, class P>
__global__ __launch_bounds__(256) void tile_kernel(P p0) {
    static_assert(WM * WN * KS == 4, "4 waves per workgroup");
    P p = p0;
    p.prepare();
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int ks = wave % KS;
    const int t = wave / KS;
    const int m0 = (blockIdx.x * WM + t / WN) * 16;
    const int n0 = (blockIdx.y * WN + t % WN) * 16;
    f32x4 acc[NB];
#pragma unroll
    for (int w = 0; w < NB; ++w) acc[w] = zero4();
    if (m0 < p.M && n0 < p.N) wave_mainloop<NB, KS>(p, m0 + (lane & 15), n0 + (lane & 15), p.K, ks, acc);
    if constexpr (KS > 1) {
        __shared__ f32x4 red[4][NB][64];
#pragma unroll
        for (int w = 0; w < NB; ++w) red[wave][w][lane] = acc[w];
        __syncthreads();
        if (ks != 0) return;
#pragma unroll
        for (int s = 1; s < KS; ++s)
#pragma unroll
            for (int w = 0; w < NB; ++w) acc[w] += red[wave + s][w][lane];
    }
    if (m0 >= p.M || n0 >= p.N) return;
    p.epilogue(m0, n0, acc);
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

// One standard normal for the 128-bit counter (Box-Muller on the first two words).
DEV float philox_normal(uint64_t seed, uint32_t c0, uint32_t c1, uint64_t c23) {
    uint32_t ctr[4] = {c0, c1, (uint32_t)c23, (uint32_t)(c23 >> 32)};
    philox4x32(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float u1 = ((float)(ctr[0] >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
    const float u2 = (float)(ctr[1] >> 8) * (1.0f / 16777216.0f);            // [0, 1)
    return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

DEV float softplusf(float a) { return fmaxf(a, 0.f) + log1pf(expf(-fabsf(a))); }
DEV float sigmoidf(float a) { return 1.0f / (1.0f + expf(-a)); }

}  // namespace vaeb
