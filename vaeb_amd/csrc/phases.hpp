// phases.hpp -- the SGVB step (VAEB.update, /root/reference/VAEB.py:408-415) as eight
// fused MFMA phases.  Each struct is one launch: operand loaders + fused epilogue.
//
//  P1 enc     h   = tanh(X W3 + b3)                                  VAEB.py:246
//  P2 heads   mu  = h W4 + b4, lv = h W5 + b5  (two accumulators)    VAEB.py:248-249
//             -> eps (Philox or injected), z = mu + exp(lv/2) eps,   VAEB.py:42-45
//                per-row KL (LB, VAEB.py:343) or prior-logQ (LA, :322-325) partials
//  P3 dechid  hd  = tanh(z W1 + b1)                                  VAEB.py:254
//  P4 decout  a2  = hd W2 + b2 (+ a6 = hd W6 + b6 Gaussian)          VAEB.py:257-263
//             -> per-row log p(x|z) partials (VAEB.py:302-313) and dA2 (+ dA6)
//  P5 dhd     dA1 = (dA2 W2^T (+ dA6 W6^T)) * (1 - hd^2)
//  P6 dz      dZ  = dA1 W1^T
//  P7 dh      [dMu|dLv] formed on the fly from dZ (sum over the L samples) and the
//             KL / LA direct terms;  dA3 = ([dMu|dLv] [W4|W5]^T) * (1 - h^2)
//  P8 wgrad   grouped TN GEMMs dW = act^T delta with a ones-row for the bias
//             gradient, fused prior (-theta, VAEB.py:386-390) + Adagrad
//             (VAEB.py:426-444), plus one workgroup that reduces the ELBO partials.
#pragma once
#include "tile_engine.hpp"

namespace vaeb {

enum : int { DEC_BERNOULLI = 0, DEC_GAUSSIAN = 1 };
enum : int { EST_LB = 0, EST_LA = 1, EST_FV = 2 };
enum : int { MODE_TRAIN = 0, MODE_EVAL = 1, MODE_RECON = 2 };
constexpr float kHalfLog2Pi = 0.91893853320467274178f;

struct StepArgs {
    int D, H, Z, L;
    int Mb;    // valid rows of this launch (batch rows of this rank)
    int Mbp;   // rows padded to 16
    int Me;    // L * Mbp decoder rows
    int dec, est, mode;
    float sc;  // loss scale: 1 (sum objective) or 1/B_global (mean objective)
    // parameters (reference order arena)
    const float *W3, *W4, *W5, *W1, *W2, *W6, *b3, *b4, *b5, *b1, *b2, *b6;
    // input rows: x = xbase + order[*cursor] * batch_stride  (order == nullptr: xbase)
    const float* xbase;
    const int* order;
    const int* cursor;
    int* cur_batch;        // written by P1 (resolved order[*cursor]); read by later phases
    int64_t batch_stride;
    int64_t row_base_mul;  // global-row id of local row i = order[*cursor]*row_base_mul + row_base_add + i
    int64_t row_base_add;
    // noise
    int eps_mode;          // 0 philox, 1 host buffer, 2 zero (reconstruct)
    uint64_t seed;
    const int64_t* step;   // Philox step counter (device)
    uint32_t domain;       // bit 0: validation; >> 1: reconstruction sample stream
    const float* eps_in;   // host-pushed [L][Mb][Z] (+ eps_in_off rows)
    int64_t eps_in_ld;     // rows per l-plane of eps_in
    // activations / deltas ([rows][cols] row-major; pad rows written as 0)
    float *h, *mu, *lv, *eps, *z, *hd, *y, *dA2, *dA6, *dA1, *dZ, *dMuLv, *dA3;
    // ELBO partials: [rows][col tiles]
    float *kl_part, *la_part, *lp_part;
    int nctZ, nctD;
    // latent slabs + per-row-block arrival counters of the folded latent phases (latent.hpp)
    float *slab_ml, *slab_dz;
    int *cnt_ml, *cnt_dz;
    // counted fixed-point accumulators of the atomic hand-off (latent.hpp: fx_*), zero
    // between launches: [Mbp][2Z] for [mu | lv], [Mbp][2Z] for [sum_l dZ | sum_l dZ eps]
    uint64_t *acc_ml, *acc_dz;
    uint64_t* dbg;         // diagnostics: per-workgroup s_memrealtime stamps (null = off)
};

// Literal FV training step: the (mu, sigma) Adagrad stream of fv_kernel rides
// enc_latent_fv_kernel's `rows` extra grid rows beyond ceil(H/16) (latent.hpp).  A kernel
// argument of its own, so StepArgs (every phase's kernarg) keeps its size.
struct FvFold {
    float *mu, *sg, *am, *as, *part;
    int64_t P;
    float lr, eps;
    int rows;
};



// P1 resolves the minibatch index from the device-side batch order; every later phase
// of the step reads the resolved copy (the cursor advances inside P8 / the optimizer).
DEV const float* x_rows_p1(const StepArgs& a) {
    return a.order ? a.xbase + (int64_t)ld_launch_const(a.cursor + kCtlNext) * a.batch_stride : a.xbase;
}
DEV const float* x_rows(const StepArgs& a) {
    return a.order ? a.xbase + (int64_t)ld_launch_const(a.cur_batch) * a.batch_stride : a.xbase;
}
DEV int64_t global_row0(const StepArgs& a) {
    return (a.order ? (int64_t)ld_launch_const(a.cur_batch) * a.row_base_mul : 0) + a.row_base_add;
}

struct NoPre {};

// ----------------------------------------------------------------------------- P1
struct PEnc {
    StepArgs a;
    const float* x;
    int M, N, K;
    rsrc_t bx, bw;
    bool vx;
    DEV void prepare() {
        x = x_rows_p1(a);
        bx = mkbuf(x, (int64_t)a.Mb * a.D * 4);
        bw = mkbuf(a.W3, (int64_t)a.D * a.H * 4);
        vx = (a.D & 3) == 0 && aligned16(x);
    }
    DEV f32x4 a4(int m, int k) const { return kc4(bx, a.D, m, k, a.Mb, a.D, vx); }
    DEV f32x4 b4(int n, int k, int) const { return mc4(bw, a.H, n, k, a.H, a.D); }
    struct Pre { float b; };
    DEV Pre prefetch(int, int n0) const {
        const int n = n0 + (threadIdx.x & 15);
        return Pre{bld(mkbuf(a.b3, (int64_t)a.H * 4), n < a.H ? (uint32_t)n * 4u : kOOB)};
    }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre& pre) const {
        const int lane = threadIdx.x & 63;
        if (a.order && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *a.cur_batch = a.cursor[kCtlNext];
        const int n = n0 + (lane & 15);
        if (n >= a.H) return;
        const float b = pre.b;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            a.h[(int64_t)m * a.H + n] = (m < a.Mb) ? ftanh(acc[0][r] + b) : 0.f;
        }
    }
};

// ----------------------------------------------------------------------------- P2
// (generic path for Z > 32; Z <= 32 uses heads_dechid_kernel in fused.hpp)
struct PHeads {
    StepArgs a;
    int M, N, K;
    rsrc_t bh, bw4, bw5;
    DEV void prepare() {
        bh = mkbuf(a.h, (int64_t)a.Mbp * a.H * 4);
        bw4 = mkbuf(a.W4, (int64_t)a.H * a.Z * 4);
        bw5 = mkbuf(a.W5, (int64_t)a.H * a.Z * 4);
    }
    DEV f32x4 a4(int m, int k) const { return kc4(bh, a.H, m, k, a.Mbp, a.H, (a.H & 3) == 0); }
    DEV f32x4 b4(int n, int k, int w) const { return mc4(w ? bw5 : bw4, a.Z, n, k, a.Z, a.H); }
    using Pre = NoPre;
    DEV Pre prefetch(int, int) const { return Pre{}; }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre&) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        const bool ncol = n < a.Z;
        const int ct = n0 >> 4;
        const int64_t grow0 = global_row0(a);
        const int64_t stp = a.step ? *a.step : 0;
        const uint64_t c23 = philox_c23(stp, a.domain);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            const bool valid = ncol && m < a.Mb;
            float mu = 0.f, lv = 0.f;
            if (valid) { mu = acc[0][r] + a.b4[n]; lv = acc[NB - 1][r] + a.b5[n]; }
            if (ncol) {
                a.mu[(int64_t)m * a.Z + n] = mu;
                a.lv[(int64_t)m * a.Z + n] = lv;
            }
            const float sd = fexp(0.5f * lv);
            float kl = valid ? 0.5f * (1.f + lv - mu * mu - fexp(lv)) : 0.f;
            for (int l = 0; l < a.L; ++l) {
                float e = 0.f;
                if (valid) {
                    if (a.eps_mode == 0)
                        e = philox_normal(a.seed, (uint32_t)(grow0 + m), (uint32_t)(l * a.Z + n), c23);
                    else if (a.eps_mode == 1)
                        e = a.eps_in[((int64_t)l * a.eps_in_ld + m) * a.Z + n];
                }
                const float z = valid ? mu + sd * e : 0.f;
                if (ncol) {
                    const int64_t o = ((int64_t)l * a.Mbp + m) * a.Z + n;
                    a.eps[o] = e;
                    a.z[o] = z;
                }
                if (a.est == EST_LA) {
                    // (-1/2 log2pi - z^2/2) - (-1/2 log2pi - lv/2 - (z-mu)^2/(2 exp lv))
                    const float d = z - mu;
                    float f = valid ? (-0.5f * z * z) - (-0.5f * lv - 0.5f * d * d / fexp(lv)) : 0.f;
                    f = sum16(f);
                    if ((lane & 15) == 0) a.la_part[((int64_t)l * a.Mbp + m) * a.nctZ + ct] = f;
                }
            }
            if (a.est != EST_LA) {
                kl = sum16(kl);
                if ((lane & 15) == 0) a.kl_part[(int64_t)m * a.nctZ + ct] = kl;
            }
        }
    }
};

// ----------------------------------------------------------------------------- P3
struct PDecHid {
    StepArgs a;
    int M, N, K;
    rsrc_t bz, bw1;
    DEV void prepare() {
        bz = mkbuf(a.z, (int64_t)a.Me * a.Z * 4);
        bw1 = mkbuf(a.W1, (int64_t)a.Z * a.H * 4);
    }
    DEV f32x4 a4(int m, int k) const { return kc4(bz, a.Z, m, k, a.Me, a.Z, (a.Z & 3) == 0); }
    DEV f32x4 b4(int n, int k, int) const { return mc4(bw1, a.H, n, k, a.H, a.Z); }
    using Pre = NoPre;
    DEV Pre prefetch(int, int) const { return Pre{}; }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre&) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        if (n >= a.H) return;
        const float b = a.b1[n];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            const bool valid = (m % a.Mbp) < a.Mb;
            a.hd[(int64_t)m * a.H + n] = valid ? ftanh(acc[0][r] + b) : 0.f;
        }
    }
};

// ----------------------------------------------------------------------------- P4
struct PDecOut {
    StepArgs a;
    const float* x;
    int M, N, K;
    rsrc_t bhd, bw2, bw6;
    DEV void prepare() { prepare_at(x_rows(a)); }
    DEV void prepare_at(const float* xr) {
        x = xr;
        bhd = mkbuf(a.hd, (int64_t)a.Me * a.H * 4);
        bw2 = mkbuf(a.W2, (int64_t)a.H * a.D * 4);
        bw6 = mkbuf(a.W6 ? a.W6 : a.W2, (int64_t)a.H * a.D * 4);
    }
    DEV f32x4 a4(int m, int k) const { return kc4(bhd, a.H, m, k, a.Me, a.H, (a.H & 3) == 0); }
    DEV f32x4 b4(int n, int k, int w) const { return mc4(w ? bw6 : bw2, a.D, n, k, a.D, a.H); }
    DEV float b1(int n, int k, int w) const {  // one element W(k, n)
        return bld(w ? bw6 : bw2, (n < a.D && k < a.H) ? (uint32_t)(k * a.D + n) * 4u : kOOB);
    }
    struct Pre { float b2, b6; f32x4 xv; };
    DEV Pre prefetch(int m0, int n0) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        const bool ncol = n < a.D;
        Pre pr;
        pr.b2 = bld(mkbuf(a.b2, (int64_t)a.D * 4), ncol ? (uint32_t)n * 4u : kOOB);
        pr.b6 = (a.dec == DEC_GAUSSIAN) ? bld(mkbuf(a.b6, (int64_t)a.D * 4), ncol ? (uint32_t)n * 4u : kOOB) : 0.f;
        const rsrc_t bxr = mkbuf(x, (int64_t)a.Mb * a.D * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = (m0 + 4 * (lane >> 4) + r) % a.Mbp;
            pr.xv[r] = bld(bxr, (ncol && i < a.Mb) ? (uint32_t)(i * a.D + n) * 4u : kOOB);
        }
        return pr;
    }
    // The operands of ONE row group r of the C/D map (rows m0 + 4 q + r): the row-parallel
    // epilogue of decout_z_kernel, where wave r finishes row group r.
    struct PreRow { float b2, b6, xv; };
    DEV PreRow prefetch_row(int m0, int n0, int r) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        const bool ncol = n < a.D;
        const int i = (m0 + 4 * (lane >> 4) + r) % a.Mbp;
        PreRow pr;
        pr.b2 = bld(mkbuf(a.b2, (int64_t)a.D * 4), ncol ? (uint32_t)n * 4u : kOOB);
        pr.b6 = (a.dec == DEC_GAUSSIAN) ? bld(mkbuf(a.b6, (int64_t)a.D * 4), ncol ? (uint32_t)n * 4u : kOOB) : 0.f;
        pr.xv = bld(mkbuf(x, (int64_t)a.Mb * a.D * 4), (ncol && i < a.Mb) ? (uint32_t)(i * a.D + n) * 4u : kOOB);
        return pr;
    }
    // Row group r: c2 = (hd W2)[m][n], c6 = (hd W6)[m][n] (Gaussian).
    DEV void epilogue_row(int m0, int n0, int r, float c2, float c6, const PreRow& pre) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        const bool ncol = n < a.D;
        const int ct = n0 >> 4;
        const float sl = a.sc / (float)a.L;
        const int m = m0 + 4 * (lane >> 4) + r;
        const int i = m % a.Mbp;
        const bool valid = ncol && i < a.Mb;
        float lp = 0.f, d2 = 0.f, d6 = 0.f, yv = 0.f, a6 = 0.f;
        if (valid) {
            const float xv = pre.xv;
            const float a2 = c2 + pre.b2;
            yv = sigmoidf(a2);
            if (a.dec == DEC_GAUSSIAN) {
                a6 = c6 + pre.b6;
                const float rr = xv - yv;
                const float e = fexp(-a6);
                lp = -kHalfLog2Pi - 0.5f * a6 - 0.5f * rr * rr * e;
                d2 = rr * e * yv * (1.f - yv) * sl;
                d6 = (-0.5f + 0.5f * rr * rr * e) * sl;
            } else {
                lp = xv * a2 - softplusf(a2);
                d2 = (xv - yv) * sl;
            }
        }
        if (ncol) {
            const int64_t o = (int64_t)m * a.D + n;
            if (a.mode == MODE_TRAIN) {
                a.dA2[o] = d2;
                if (a.dec == DEC_GAUSSIAN) a.dA6[o] = d6;
            } else if (a.mode == MODE_RECON) {
                a.y[o] = yv;
                // the decoder's log-sigma head (VAEB.py:258, freyFace.py:178): the dA6
                // plane is free outside training
                if (a.dec == DEC_GAUSSIAN) a.dA6[o] = a6;
            }
        }
        lp = sum16(lp);
        if ((lane & 15) == 0) a.lp_part[(int64_t)m * a.nctD + ct] = lp;
    }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre& pre) const {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            epilogue_row(m0, n0, r, acc[0][r], acc[NB - 1][r], PreRow{pre.b2, pre.b6, pre.xv[r]});
    }
};

// ----------------------------------------------------------------------------- P5
// [dA2 | dA6] and [W2 | W6] are each ONE allocation (dA6 = dA2 + dplane elements, W6 = W2 +
// H D in the arena), so both K halves go through one buffer descriptor and a per-lane
// offset select: the loaders are branch-free.  (With a descriptor chosen per K half in a
// branch -- and the 16-byte form chosen at run time -- hipcc drained vmcnt inside every
// chunk's branch, serialising the wave's eight chunk loads into eight round trips.)
// V (host-chosen): D % 4 == 0 and 16-byte aligned dA2 / W2: one 16-byte load per operand.
template <bool V>
struct PDhdT {
    StepArgs a;
    int M, N, K;  // K = D (Bernoulli) or Dp + D (Gaussian: [dA2|dA6] . [W2|W6]^T, Dp = D rounded to 4)
    int Dp;
    int64_t dplane, wplane;   // elements from dA2 to dA6 / from W2 to W6 (0: Bernoulli)
    rsrc_t bd, bw;
    DEV void prepare() {
        Dp = (a.D + 3) & ~3;
        const bool gs = a.dec == DEC_GAUSSIAN;
        dplane = gs ? (int64_t)(a.dA6 - a.dA2) : 0;
        wplane = gs ? (int64_t)(a.W6 - a.W2) : 0;
        bd = mkbuf(a.dA2, (dplane + (int64_t)a.Me * a.D) * 4);
        bw = mkbuf(a.W2, (wplane + (int64_t)a.H * a.D) * 4);
    }
    // element (r, k) of the K-concatenated operand: k in [Dp, Dp + D) is the Gaussian half
    DEV f32x4 ld(rsrc_t b, int64_t plane, int r, int rlim, int k) const {
        const bool hi = k >= Dp;
        const int kk = hi ? k - Dp : k;
        const uint32_t base = (uint32_t)((hi ? plane : 0) + (int64_t)r * a.D + kk) * 4u;
        const bool rok = r < rlim && (!hi || plane != 0);
        if (V) return bld4(b, (rok && kk < a.D) ? base : kOOB);
        f32x4 v;
#pragma unroll
        for (int s = 0; s < 4; ++s) v[s] = bld(b, (rok && kk + s < a.D) ? base + 4u * s : kOOB);
        return v;
    }
    DEV f32x4 a4(int m, int k) const { return ld(bd, dplane, m, a.Me, k); }
    DEV f32x4 b4(int n, int k, int) const { return ld(bw, wplane, n, a.H, k); }
    struct Pre { f32x4 hd; };
    DEV Pre prefetch(int m0, int n0) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        const rsrc_t b = mkbuf(a.hd, (int64_t)a.Me * a.H * 4);
        Pre pr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            pr.hd[r] = bld(b, (n < a.H && m < a.Me) ? (uint32_t)(m * a.H + n) * 4u : kOOB);
        }
        return pr;
    }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre& pre) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        if (n >= a.H) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            const int64_t o = (int64_t)m * a.H + n;
            const float hd = pre.hd[r];
            a.dA1[o] = ((m % a.Mbp) < a.Mb) ? acc[0][r] * (1.f - hd * hd) : 0.f;
        }
    }
};

// ----------------------------------------------------------------------------- P6
// (generic path for Z > 32; Z <= 32 uses dz_dh_kernel in fused.hpp)
struct PDz {
    StepArgs a;
    int M, N, K;
    rsrc_t bd1, bw1;
    DEV void prepare() {
        bd1 = mkbuf(a.dA1, (int64_t)a.Me * a.H * 4);
        bw1 = mkbuf(a.W1, (int64_t)a.Z * a.H * 4);
    }
    DEV f32x4 a4(int m, int k) const { return kc4(bd1, a.H, m, k, a.Me, a.H, (a.H & 3) == 0); }
    DEV f32x4 b4(int n, int k, int) const { return kc4(bw1, a.H, n, k, a.Z, a.H, (a.H & 3) == 0 && aligned16(a.W1)); }
    using Pre = NoPre;
    DEV Pre prefetch(int, int) const { return Pre{}; }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre&) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        if (n >= a.Z) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            a.dZ[(int64_t)m * a.Z + n] = ((m % a.Mbp) < a.Mb) ? acc[0][r] : 0.f;
        }
    }
};

// ----------------------------------------------------------------------------- P7
struct PDh {
    StepArgs a;
    int M, N, K;  // K = 2Z
    rsrc_t bw4, bw5;
    DEV void prepare() {
        bw4 = mkbuf(a.W4, (int64_t)a.H * a.Z * 4);
        bw5 = mkbuf(a.W5, (int64_t)a.H * a.Z * 4);
    }
    // [dMu | dLv](i, k) from dZ, mu, lv, eps, z (LA variant).
    DEV float dmulv(int i, int k) const {
        const int Z = a.Z;
        const bool isv = k >= Z;
        const int j = isv ? k - Z : k;
        const int64_t o = (int64_t)i * Z + j;
        const float mu = a.mu[o], lv = a.lv[o];
        const float sd = fexp(0.5f * lv);
        const float sl = a.sc / (float)a.L;
        float g = 0.f, t = 0.f;
        for (int l = 0; l < a.L; ++l) {
            const int64_t ol = ((int64_t)l * a.Mbp + i) * Z + j;
            const float dz = a.dZ[ol];
            const float e = a.eps[ol];
            if (!isv) {
                g += dz;
                if (a.est == EST_LA) t += -a.z[ol];
            } else {
                g += dz * 0.5f * sd * e;
                if (a.est == EST_LA) t += 0.5f - 0.5f * a.z[ol] * sd * e;
            }
        }
        if (a.est == EST_LA) return g + sl * t;
        return isv ? g + a.sc * 0.5f * (1.f - fexp(lv)) : g - a.sc * mu;
    }
    DEV f32x4 a4(int m, int k) const {
        f32x4 v = zero4();
        const int K2 = 2 * a.Z;
        if (m < a.Mb) {
            if (k + 0 < K2) v.x = dmulv(m, k + 0);
            if (k + 1 < K2) v.y = dmulv(m, k + 1);
            if (k + 2 < K2) v.z = dmulv(m, k + 2);
            if (k + 3 < K2) v.w = dmulv(m, k + 3);
        }
        // the column-tile-0 wave publishes [dMu|dLv] (pad rows as 0) for the
        // weight-gradient phase
        if (m < a.Mbp && blockIdx.y == 0 && ((threadIdx.x >> 6) == 0)) {
            float* o = a.dMuLv + (int64_t)m * K2;
            if (k + 0 < K2) o[k + 0] = v.x;
            if (k + 1 < K2) o[k + 1] = v.y;
            if (k + 2 < K2) o[k + 2] = v.z;
            if (k + 3 < K2) o[k + 3] = v.w;
        }
        return v;
    }
    // B(k, n) = [W4 | W5]^T: both halves loaded with out-of-range offsets for the other.
    DEV f32x4 b4(int n, int k, int) const {
        const int Z = a.Z;
        f32x4 v;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kk = k + s;
            const bool ok = n < a.H;
            const float w4 = bld(bw4, (ok && kk < Z) ? (uint32_t)(n * Z + kk) * 4u : kOOB);
            const float w5 = bld(bw5, (ok && kk >= Z && kk < 2 * Z) ? (uint32_t)(n * Z + kk - Z) * 4u : kOOB);
            v[s] = w4 + w5;
        }
        return v;
    }
    using Pre = NoPre;
    DEV Pre prefetch(int, int) const { return Pre{}; }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre&) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        if (n >= a.H) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            const int64_t o = (int64_t)m * a.H + n;
            const float h = a.h[o];
            a.dA3[o] = (m < a.Mb) ? acc[0][r] * (1.f - h * h) : 0.f;
        }
    }
};

}  // namespace vaeb
