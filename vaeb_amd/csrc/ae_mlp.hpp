// ae_mlp.hpp -- fp32 MFMA layer-stack kernels for the degenerate-vae deterministic
// autoencoder (/root/reference/degenerate-vae/ae.py:41-117, mlp.py:36-91, logpdf.py:46-114,
// infalg.py:148-164), on the same tile engine as the VAEB step (tile_engine.hpp).
//
// One training call train(idx) (ae.py:82-89) on the gathered rows X = Xtr[idx]:
//   forward, per layer:   out = f(in W + b)            PAeFwd (mode ACT / LINEAR)
//                         Z layer linear (ae.py:49)
//   output (ae.py:58-73): binary  P = sigmoid(a), loglik += Y log(P+1e-7) + (1-Y) log(1-P+1e-7)
//                         cont    mu = sigmoid(a_mu), ls2 = a_ls2,
//                                 loglik += -1/2 (log 2 pi + ls2 + (Y-mu)^2 e^-ls2)
//                         fused with the output deltas dlogjoint/da     PAeFwd (mode OUT_*)
//   backward, per layer:  din = (dout W^T) * f'(h)      PAeBwd (mode DACT)
//                         dZ  = dout W^T - Z            PAeBwd (mode ZPRIOR: N(0,1) prior on Z)
//   weight gradients:     [in | 1]^T dout (ones row = bias gradient), prior -theta/s2 and
//                         AdaGrad (infalg.py:155-161) in the epilogue   PAeWgrad
// The first layer's A operand is gathered on the fly through idx (no copy of Xtr[idx]).
// Every weight is updated only after the last kernel of the step that reads it, so the
// update is simultaneous in the Theano sense.
#pragma once
#include "tile_engine.hpp"

namespace vaeb {
namespace ae {

enum : int { ACT_TANH = 0, ACT_SIGMOID = 1, ACT_RELU = 2 };
enum : int { F_ACT = 0, F_LINEAR = 1, F_OUT_BIN = 2, F_OUT_CONT = 3 };
enum : int { B_DACT = 0, B_ZPRIOR = 1 };
constexpr float kEpsLog = 1e-7f;   // logpdf.py:86
constexpr float kHalfLog2Pi = 0.91893853320467274178f;

struct Dbg { uint64_t* dbg; };

DEV float act_f(int act, float v) {
    if (act == ACT_TANH) return ftanh(v);
    if (act == ACT_SIGMOID) return sigmoidf(v);
    return fmaxf(v, 0.f);
}
DEV float dact_f(int act, float h) {   // in terms of the stored activation h
    if (act == ACT_TANH) return 1.f - h * h;
    if (act == ACT_SIGMOID) return h * (1.f - h);
    return h > 0.f ? 1.f : 0.f;
}

// element (r, k) of a row-major [rows x ld] matrix, 0 outside [0, rlim) x [0, klim)
DEV float el(rsrc_t b, int ld, int r, int k, int rlim, int klim) {
    return bld(b, (r < rlim && k < klim && r >= 0) ? (uint32_t)(r * ld + k) * 4u : kOOB);
}

// ---------------------------------------------------------------- forward layer
struct PAeFwd {
    Dbg a;
    int M, N, K;
    const float* in; int ldin; int in_rows; const int* idx;   // idx: gathered input rows
    const float *W, *W2, *b, *b2;                             // W [K x N] (W2: Wlogs2)
    int mode, act;
    float *out, *out2;                                        // activations / Xpr (+ ls2)
    const float* Y; const int* yidx; int ldy; int y_rows;     // observations (output layer)
    float *dA, *dA2;                                          // output deltas
    float* llpart; int nct;                                   // [M][nct] log-lik partials
    rsrc_t bin, bw, bw2, by;
    DEV void prepare() {
        bin = mkbuf(in, (int64_t)in_rows * ldin * 4);
        bw = mkbuf(W, (int64_t)K * N * 4);
        bw2 = mkbuf(W2 ? W2 : W, (int64_t)K * N * 4);
        by = mkbuf(Y ? Y : in, (int64_t)(Y ? y_rows : in_rows) * (Y ? ldy : ldin) * 4);
    }
    DEV int row_of(int m) const { return m < M ? (idx ? idx[m] : m) : -1; }
    DEV f32x4 a4(int m, int k) const {
        const int r = row_of(m);
        f32x4 v;
        v.x = el(bin, ldin, r, k + 0, in_rows, K);
        v.y = el(bin, ldin, r, k + 1, in_rows, K);
        v.z = el(bin, ldin, r, k + 2, in_rows, K);
        v.w = el(bin, ldin, r, k + 3, in_rows, K);
        return v;
    }
    DEV f32x4 b4(int n, int k, int w) const { return mc4(w ? bw2 : bw, N, n, k, N, K); }
    using Pre = NoPre;
    DEV Pre prefetch(int, int) const { return Pre{}; }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre&) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        const bool nok = n < N;
        const float bb = nok ? b[n] : 0.f;
        const float bb2 = (nok && b2) ? b2[n] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            const bool ok = nok && m < M;
            const float v = acc[0][r] + bb;
            if (mode == F_ACT || mode == F_LINEAR) {
                if (ok) out[(int64_t)m * N + n] = (mode == F_ACT) ? act_f(act, v) : v;
                continue;
            }
            if (!Y) {   // predictions only (reconstruct / decode): Xpr (+ ls2)
                if (ok) out[(int64_t)m * N + n] = sigmoidf(v);
                if constexpr (NB > 1)
                    if (ok) out2[(int64_t)m * N + n] = acc[1][r] + bb2;
                continue;
            }
            const int yr = ok ? (yidx ? yidx[m] : m) : 0;
            const float y = ok ? Y[(int64_t)yr * ldy + n] : 0.f;
            float ll = 0.f;
            if (mode == F_OUT_BIN) {
                const float P = sigmoidf(v);
                ll = y * flog(P + kEpsLog) + (1.f - y) * flog(1.f - P + kEpsLog);
                const float dP = y / (P + kEpsLog) - (1.f - y) / (1.f - P + kEpsLog);
                if (ok) {
                    out[(int64_t)m * N + n] = P;
                    dA[(int64_t)m * N + n] = dP * P * (1.f - P);
                }
            } else {
                float ls2 = bb2;
                if constexpr (NB > 1) ls2 += acc[1][r];
                const float mu = sigmoidf(v);
                const float rr = y - mu, e = fexp(-ls2);
                ll = -kHalfLog2Pi - 0.5f * ls2 - 0.5f * rr * rr * e;
                if (ok) {
                    out[(int64_t)m * N + n] = mu;
                    out2[(int64_t)m * N + n] = ls2;
                    dA[(int64_t)m * N + n] = rr * e * mu * (1.f - mu);
                    dA2[(int64_t)m * N + n] = -0.5f + 0.5f * rr * rr * e;
                }
            }
            const float s = sum16(ok ? ll : 0.f);
            if ((lane & 15) == 0 && m < M) llpart[(int64_t)m * nct + n0 / 16] = s;
        }
    }
};

// ---------------------------------------------------------------- backward (data) layer
// din[M x N] = [dout | dout2] [W | W2]^T  (K = K1 or 2 K1), then * f'(h) or - h (Z prior).
struct PAeBwd {
    Dbg a;
    int M, N, K;
    const float *dout, *dout2; int K1;
    const float *W, *W2;             // [N x K1] each (row n = this layer's input unit)
    const float* h; int mode, act;   // h [M x N]: activation (DACT) or Z (ZPRIOR)
    float* din;
    rsrc_t bd, bd2, bw, bw2;
    DEV void prepare() {
        bd = mkbuf(dout, (int64_t)M * K1 * 4);
        bd2 = mkbuf(dout2 ? dout2 : dout, (int64_t)M * K1 * 4);
        bw = mkbuf(W, (int64_t)N * K1 * 4);
        bw2 = mkbuf(W2 ? W2 : W, (int64_t)N * K1 * 4);
    }
    DEV float src(rsrc_t b1, rsrc_t b2, int r, int k, int rl) const {
        return k < K1 ? el(b1, K1, r, k, rl, K1) : el(b2, K1, r, k - K1, rl, K1);
    }
    DEV f32x4 a4(int m, int k) const {
        f32x4 v;
        v.x = src(bd, bd2, m, k + 0, M);
        v.y = src(bd, bd2, m, k + 1, M);
        v.z = src(bd, bd2, m, k + 2, M);
        v.w = src(bd, bd2, m, k + 3, M);
        if (k + 0 >= K) v.x = 0.f;
        if (k + 1 >= K) v.y = 0.f;
        if (k + 2 >= K) v.z = 0.f;
        if (k + 3 >= K) v.w = 0.f;
        return v;
    }
    DEV f32x4 b4(int n, int k, int) const {
        f32x4 v;
        v.x = src(bw, bw2, n, k + 0, N);
        v.y = src(bw, bw2, n, k + 1, N);
        v.z = src(bw, bw2, n, k + 2, N);
        v.w = src(bw, bw2, n, k + 3, N);
        return v;
    }
    using Pre = NoPre;
    DEV Pre prefetch(int, int) const { return Pre{}; }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre&) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        if (n >= N) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            if (m >= M) continue;
            const float hv = h[(int64_t)m * N + n];
            din[(int64_t)m * N + n] = (mode == B_DACT) ? acc[0][r] * dact_f(act, hv) : acc[0][r] - hv;
        }
    }
};

// ---------------------------------------------------------------- weight gradient + AdaGrad
// C[Kin + 1 x N] = [in | 1]^T dout over the M batch rows (row Kin = the bias gradient),
// g = C - theta / s2 (mlp.py:87-91 prior), acc += g^2, theta += eta g / (sqrt(acc) + 1e-6).
struct PAeWgrad {
    Dbg a;
    int M, N, K;                     // M = Kin + 1, N = out width, K = batch rows
    const float* in; int ldin; int in_rows; const int* idx; int Kin;
    const float* dout;
    float *theta, *accum; int64_t offW, offb;
    float eta, inv_s2;
    rsrc_t bin, bd;
    DEV void prepare() {
        bin = mkbuf(in, (int64_t)in_rows * ldin * 4);
        bd = mkbuf(dout, (int64_t)K * N * 4);
    }
    DEV float ina(int m, int k) const {
        if (k >= K) return 0.f;
        if (m == Kin) return 1.f;
        const int r = idx ? idx[k] : k;
        return el(bin, ldin, r, m, in_rows, Kin);
    }
    DEV f32x4 a4(int m, int k) const {
        f32x4 v;
        v.x = ina(m, k + 0);
        v.y = ina(m, k + 1);
        v.z = ina(m, k + 2);
        v.w = ina(m, k + 3);
        return v;
    }
    DEV f32x4 b4(int n, int k, int) const { return mc4(bd, N, n, k, N, K); }
    using Pre = NoPre;
    DEV Pre prefetch(int, int) const { return Pre{}; }
    template <int NB>
    DEV void epilogue(int m0, int n0, const f32x4 (&acc)[NB], const Pre&) const {
        const int lane = threadIdx.x & 63;
        const int n = n0 + (lane & 15);
        if (n >= N) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * (lane >> 4) + r;
            if (m > Kin) continue;
            const int64_t i = (m == Kin) ? offb + n : offW + (int64_t)m * N + n;
            const float th = theta[i];
            const float g = acc[0][r] - th * inv_s2;
            const float ac = accum[i] + g * g;
            accum[i] = ac;
            theta[i] = th + eta * g / (sqrtf(ac) + 1e-6f);
        }
    }
};

// Log-likelihood of the step: fixed-order fp64 sum of the [M][nct] partials -> out[slot]
// (= loglik / M, the value train() returns, ae.py:86).
__global__ __launch_bounds__(256) void ae_loglik_kernel(const float* part, int64_t n, int M, float* out, int slot) {
    __shared__ double sh[256];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 256) s += part[i];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[slot] = (float)(sh[0] / (double)M);
}

}  // namespace ae
}  // namespace vaeb
