// kernels_aux.hpp -- the weight-gradient / optimizer end of the SGVB step and the
// reductions (/root/reference/VAEB.py:385-444).
#pragma once
#include "fused.hpp"

namespace vaeb {

// ----------------------------------------------------------------- ELBO reduction
struct ElboArgs {
    const float* lp_part; int64_t n_lp;   // [Me][nctD] per-row log p(x|z) partials
    const float* kl_part; int64_t n_kl;   // [Mbp][nctZ] KL partials (LB / FV) or
                                          // [Me][nctZ] prior-logQ partials (LA)
    const float* fv_part; int64_t n_fv;   // FV thetaPrior partials (per workgroup)
    int L, est;
    double data_mul;      // FV: x.shape[0] (VAEB.py:364); else 1
    double inv_bglob;     // 1 / B_global
    float* elbo_out;      // SGVB / B_global of the last step
    double* epoch;        // [0] += SGVB / B_global, [1] += 1
    float* dp_slot;       // DP: write the local SGVB here (reduced with the gradients)
    double* eval_acc;     // validate: [0] += data term, [1] += thetaPrior
    int* cursor;          // advanced once per step
    int64_t* step;
};

DEV double block_sum256(double v, double* sh) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
#pragma unroll
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) sh[t] += sh[t + o];
        __syncthreads();
    }
    const double r = sh[0];
    __syncthreads();
    return r;
}

// Deterministic (fixed-order) reduction by one 256-thread workgroup.
DEV void elbo_reduce(const ElboArgs& e) {
    __shared__ double sh[256];
    double lp = 0, kl = 0, fv = 0;
    for (int64_t i = threadIdx.x; i < e.n_lp; i += 256) lp += e.lp_part[i];
    for (int64_t i = threadIdx.x; i < e.n_kl; i += 256) kl += e.kl_part[i];
    for (int64_t i = threadIdx.x; i < e.n_fv; i += 256) fv += e.fv_part[i];
    lp = block_sum256(lp, sh);
    kl = block_sum256(kl, sh);
    fv = block_sum256(fv, sh);
    if (threadIdx.x != 0) return;
    // LB: sum logp / L + sum KL (VAEB.py:339-344); LA: (sum logp + sum(prior-logQ)) / L
    // (VAEB.py:327-328); FV: B * (sum logp + sum KL) + thetaPrior (VAEB.py:364).
    const double data = (e.est == EST_LA) ? (lp + kl) / e.L : lp / e.L + kl;
    const double sg = (e.est == EST_FV) ? e.data_mul * data + fv : data;
    if (e.eval_acc) { e.eval_acc[0] += data; e.eval_acc[1] = fv; }
    if (e.dp_slot) {
        *e.dp_slot = (float)sg;
    } else if (e.elbo_out) {
        const double v = sg * e.inv_bglob;
        *e.elbo_out = (float)v;
        e.epoch[0] += v;
        e.epoch[1] += 1.0;
    }
    if (e.cursor) *e.cursor += 1;
    if (e.step) *e.step += 1;
}

__global__ __launch_bounds__(256) void elbo_kernel(ElboArgs e) { elbo_reduce(e); }

// ----------------------------------------------------------------- optimizer rule
struct OptArgs {
    float* theta; float* acc; float* grad;
    float lr, eps, prior, decay;  // decay = lr*eps for the mean_map variant, else 0
    int update, store_grad;
};

// VAEB.getUpdates (VAEB.py:438-442) on one element, prior folded in (VAEB.py:389-390):
//   g = dSGVB/dtheta - prior*theta;  acc += g^2;  theta += lr*g/(sqrt(acc)+eps) [- decay*theta^2]
DEV void opt_apply(const OptArgs& o, int64_t idx, float dsg) {
    if (o.store_grad) o.grad[idx] = dsg;
    if (!o.update) return;
    const float th = o.theta[idx];
    const float g = dsg - o.prior * th;
    const float a = o.acc[idx] + g * g;
    o.acc[idx] = a;
    o.theta[idx] = th + o.lr * g / (sqrtf(a) + o.eps) - o.decay * th * th;
}

// ----------------------------------------------------------------- P8 weight gradients
// C[i][j] = sum_k At[k][i] * Bm[k][j] over the minibatch rows k, with row i == rowsW the
// all-ones row, so the bias gradient (the column sum of the delta) is the last row.
struct WGroup {
    const float* at; int ld_at; int klim_at; int at_is_x;
    int rowsW;
    const float* bm0; const float* bm1; int ld_b; int nb;
    int N, K;
    int64_t offW0, offb0, offW1, offb1;
    int tiles_n, wg_begin, wg_end;
};

struct WGradArgs {
    WGroup g[4];
    int ngroups, total_wgs;
    OptArgs opt;
    ElboArgs elbo;
    const float* xbase; const int* cur_batch; int64_t batch_stride;
    int64_t P;
    uint64_t* dbg;
};

struct WGProb {
    const WGroup* g;
    rsrc_t bat, bb0, bb1;
    DEV f32x4 a4(int i, int k) const {
        f32x4 v = mc4(bat, g->ld_at, i, k, g->rowsW, g->klim_at);
        const bool one = i == g->rowsW;  // the all-ones row (bias gradient), branch-free
        v.x = one ? ((k + 0 < g->K) ? 1.f : 0.f) : v.x;
        v.y = one ? ((k + 1 < g->K) ? 1.f : 0.f) : v.y;
        v.z = one ? ((k + 2 < g->K) ? 1.f : 0.f) : v.z;
        v.w = one ? ((k + 3 < g->K) ? 1.f : 0.f) : v.w;
        return v;
    }
    DEV f32x4 b4(int j, int k, int w) const { return mc4(w ? bb1 : bb0, g->ld_b, j, k, g->N, g->K); }
};

template <int NB>
DEV void wgrad_tile(const WGradArgs& p, const WGroup& g, const float* at, int m0, int n0, int64_t P) {
    f32x4 acc[NB];
#pragma unroll
    for (int w = 0; w < NB; ++w) acc[w] = zero4();
    const int lane = threadIdx.x & 63;
    const int j = n0 + (lane & 15);
    const rsrc_t bth = mkbuf(p.opt.theta, P * 4), bac = mkbuf(p.opt.acc, P * 4), bgr = mkbuf(p.opt.grad, P * 4);
    // prefetch theta / acc of this lane's outputs so the optimizer epilogue does not pay
    // a second memory round trip after the MFMA chain (byte offsets; kOOB = masked)
    uint32_t off[4][NB];
    float th[4][NB], ac[4][NB];
    const bool upd = p.opt.update != 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = m0 + 4 * (lane >> 4) + r;
        const bool ok = j < g.N && i <= g.rowsW;
#pragma unroll
        for (int w = 0; w < NB; ++w) {
            const int64_t idx = (i < g.rowsW) ? (w ? g.offW1 : g.offW0) + (int64_t)i * g.N + j : (w ? g.offb1 : g.offb0) + j;
            off[r][w] = ok ? (uint32_t)idx * 4u : kOOB;
            th[r][w] = upd ? bld(bth, off[r][w]) : 0.f;
            ac[r][w] = upd ? bld(bac, off[r][w]) : 0.f;
        }
    }
    WGProb prob{&g, mkbuf(at, (int64_t)g.klim_at * g.ld_at * 4), mkbuf(g.bm0, (int64_t)g.K * g.ld_b * 4),
                mkbuf(g.bm1 ? g.bm1 : g.bm0, (int64_t)g.K * g.ld_b * 4)};
    if (m0 <= g.rowsW && n0 < g.N) wave_mainloop<NB, 1, 8>(prob, m0 + (lane & 15), n0 + (lane & 15), g.K, 0, acc);
    if (p.dbg && threadIdx.x == 0) p.dbg[blockIdx.x * 8 + 1] = __builtin_amdgcn_s_memrealtime();
    // out-of-range byte offsets make the masked buffer stores no-ops
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int w = 0; w < NB; ++w) {
            const float dsg = acc[w][r];
            if (p.opt.store_grad) bst(bgr, off[r][w], dsg);
            if (upd) {
                const float t0 = th[r][w];
                const float g2 = dsg - p.opt.prior * t0;
                const float a2 = ac[r][w] + g2 * g2;
                bst(bac, off[r][w], a2);
                bst(bth, off[r][w], t0 + p.opt.lr * g2 / (sqrtf(a2) + p.opt.eps) - p.opt.decay * t0 * t0);
            }
        }
}

__global__ __launch_bounds__(256) void wgrad_kernel(WGradArgs p) {
    const int bid = blockIdx.x;
    if (p.dbg && threadIdx.x == 0) p.dbg[bid * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    if (bid >= p.total_wgs) {  // the extra workgroup: ELBO of this step
        elbo_reduce(p.elbo);
        return;
    }
    int gi = 0;
#pragma unroll
    for (int t = 1; t < 4; ++t)
        if (t < p.ngroups && bid >= p.g[t].wg_begin) gi = t;
    const WGroup& g = p.g[gi];
    const float* at = g.at_is_x ? p.xbase + (int64_t)(*p.cur_batch) * p.batch_stride : g.at;
    const int lt = bid - g.wg_begin;
    const int wave = threadIdx.x >> 6;
    const int m0 = ((lt / g.tiles_n) * 2 + (wave >> 1)) * 16;
    const int n0 = ((lt % g.tiles_n) * 2 + (wave & 1)) * 16;
    if (g.nb == 2) wgrad_tile<2>(p, g, at, m0, n0, p.P);
    else wgrad_tile<1>(p, g, at, m0, n0, p.P);
    if (p.dbg && threadIdx.x == 0) p.dbg[bid * 8 + 3] = __builtin_amdgcn_s_memrealtime();
}

// ----------------------------------------------------------------- DP optimizer
// After the RCCL all-reduce of [grad arena | SGVB]: replicated Adagrad with the prior
// added once (so every rank applies the identical update).
__global__ __launch_bounds__(256) void adagrad_kernel(OptArgs o, int64_t P, ElboArgs e) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    OptArgs u = o;
    u.store_grad = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < P; i += stride) opt_apply(u, i, o.grad[i]);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const double v = (double)o.grad[P] * e.inv_bglob;
        *e.elbo_out = (float)v;
        e.epoch[0] += v;
        e.epoch[1] += 1.0;
        *e.cursor += 1;
        *e.step += 1;
    }
}

// ----------------------------------------------------------------- full variational
// Literal --full_varational update (VAEB.py:117-125, 349-367, 392-393, 426-444):
// g_mu = -2 mu, g_sigma = 1/sigma - 2 sigma; thetaPrior partials from pre-update values.
__global__ __launch_bounds__(256) void fv_kernel(float* mu, float* sg, float* am, float* as, int64_t P,
                                                 float lr, float eps, int update, float* part) {
    __shared__ double sh[256];
    double tp = 0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < P; i += stride) {
        const float m = mu[i], s = sg[i];
        tp += 0.5 * (1.0 + (double)logf(s * s) - (double)m * m - (double)s * s);
        if (update) {
            const float gm = -2.f * m;
            const float gs = 1.f / s - 2.f * s;
            const float a1 = am[i] + gm * gm;
            const float a2 = as[i] + gs * gs;
            am[i] = a1;
            as[i] = a2;
            mu[i] = m + lr * gm / (sqrtf(a1) + eps);
            sg[i] = s + lr * gs / (sqrtf(a2) + eps);
        }
    }
    tp = block_sum256(tp, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = (float)tp;
}

}  // namespace vaeb
