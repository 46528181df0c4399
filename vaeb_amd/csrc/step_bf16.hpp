// step_bf16.hpp -- the non-GEMM kernels of the bf16 large-batch SGVB step.
//
// The step (VAEB.update, /root/reference/VAEB.py:408-415) on the bf16 engine is
//   enc     h     = tanh(X W3 + b3)                      GEMM, KC x KO   VAEB.py:246
//   heads   [mu|lv] slabs = h [W4|W5]                    GEMM split-K    VAEB.py:248-249
//   latent  mu, lv (+bias), eps, z, KL / LA row terms    latent_fwd      VAEB.py:41-47, 315-346
//   dechid  hd    = tanh(z W1 + b1)                      GEMM            VAEB.py:254
//   decout  log p(x|z) row partials, dA2 (| dA6)         GEMM + EpiDecOut VAEB.py:257-313
//   dhd     dA1   = ([dA2|dA6] [W2|W6]^T) (1 - hd^2)     GEMM KC x KC
//   dW26    Adagrad([hd]^T [dA2|dA6])                    GEMM KO x KO + EpiAdagrad
//   dz      dZ slabs = dA1 W1^T                          GEMM split-K
//   dW1     slabs z^T dA1 -> wreduce_opt                 GEMM split-K
//   latentb [dMu|dLv] (sum over l), b4/b5 column sums    latent_bwd      
//   dh      dA3   = ([dMu|dLv] [W4|W5]^T) (1 - h^2)      GEMM KC x KC
//   dW45    slabs h^T [dMu|dLv] -> wreduce_opt           GEMM split-K
//   dW3     Adagrad(X^T dA3)                             GEMM KO x KO + EpiAdagrad
//   bias    bias gradients from the column partials, Adagrad, ELBO reduce, cursor++
// Parameters keep fp32 masters in the reference-order arena (ping-pong, as the fp32
// path) plus a bf16 "shadow" arena in GEMM layout that the optimizer rewrites each step:
//   W3 [D x H] | W45 [H x 2Z] (row h = [W4 row h | W5 row h]) | W1 [Z x H] |
//   W26 [H x Dn] (Bernoulli: W2; Gaussian: W2 / W6 interleaved in 32-column groups).
// Included twice by h16_engines.hpp (namespace VAEB_H16NS = bf / hf), after gemm_bf16.hpp.
#include "kernels_aux.hpp"

namespace vaeb {
namespace VAEB_H16NS {

using ::vaeb::h16c::BfState;

using ::vaeb::h16c::ShadowMap;

// Sharded DP (vaeb_hip.hip dp_reduce_update): after the all-gather of theta', the bf16 shadow
// entries of the elements other ranks updated
__global__ __launch_bounds__(256) void shadow_runs_kernel(const float* th, bf16_t* sh, ShadowMap m, DpRange r) {
    const int64_t stride = (int64_t)gridDim.x * 256, n = r.total();
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n; v += stride) {
        const int64_t i = r.at(v), si = m.at(i);
        if (si >= 0) sh[si] = (bf16_t)f2bf(th[i]);
    }
}

// diagnostics (vaeb_get_shadow): the shadow entries of the weight elements, in arena order
__global__ __launch_bounds__(256) void shadow_gather_kernel(const bf16_t* sh, bf16_t* out, ShadowMap m) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m.nweights; i += stride) out[i] = sh[m.at(i)];
}

// theta (fp32 arena) -> bf16 shadow
__global__ __launch_bounds__(256) void make_shadow_kernel(const float* th, bf16_t* sh, ShadowMap m) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m.nweights; i += stride)
        sh[m.at(i)] = (bf16_t)f2bf(th[i]);
}

// fp32 rows -> bf16 (dataset upload)
__global__ __launch_bounds__(256) void to_bf16_kernel(const float* in, bf16_t* out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) out[i] = (bf16_t)f2bf(in[i]);
}

struct LatentArgs {
    int M, Z, L, est, mode;        // M rows of this launch; mode: MODE_TRAIN / EVAL / RECON
    float sc;
    const float* ml_slab; int nslab;   // heads split-K slabs [nslab][M][2Z]
    const float *b4, *b5;
    float *mu, *lv, *eps;              // [M][Z], [M][Z], [L][M][Z]
    bf16_t* z;                         // [L][M][Z]
    float* kl_part;                    // LB: [M]; LA: [L][M]
    // noise (VAEB.py:41-47): Philox keyed by (seed, step, global row, l*Z + j)
    int eps_mode; uint64_t seed; const int64_t* step; uint32_t domain;
    const float* eps_in; int64_t eps_in_ld;
    BatchRef rows; int64_t row_base_add;   // global row of local row 0 = batch*mul + add
    int64_t row_base_mul;
    // backward
    const float* dz_slab; int ndz;     // [ndz][L*M][Z]
    bf16_t* dmulv;                     // [M][2Z]
    float* colpart;                    // [ceil(M/64)][2Z]
};

// Fixed-order sum of n fp32 split-K slab values (v[s * stride + off], s = 0..n-1) added to
// `init`: the loads go out in groups of 8 through a buffer descriptor (slot s >= n reads 0
// from the hardware range check), so a group is ONE memory round trip instead of n
// dependent ones, and the running sum keeps the slab order.
DEV float slab_sum(rsrc_t b, uint32_t off, uint32_t stride, int n, bool ok, float init) {
    float acc = init;
    for (int s0 = 0; s0 < n; s0 += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            v[u] = bld(b, (ok && s0 + u < n) ? off + (uint32_t)(s0 + u) * stride : kOOB);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    return acc;
}

// One wave per row: mu / lv from the heads slabs (fixed-order sum) + bias; eps; z; the
// per-row KL (LB, VAEB.py:343) or, per sample, prior - logQ (LA, VAEB.py:322-325).
__global__ __launch_bounds__(256) void latent_fwd_kernel(LatentArgs a) {
    const int lane = threadIdx.x & 63;
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= a.M) return;
    const int Z = a.Z, Z2 = 2 * Z;
    const int64_t brow = a.rows.order ? (int64_t)a.rows.order[*a.rows.cursor] : 0;
    const int64_t grow = brow * a.row_base_mul + a.row_base_add + m;
    const uint64_t c23 = philox_c23(*a.step, a.domain);
    const rsrc_t bsl = mkbuf(a.ml_slab, (int64_t)a.nslab * a.M * Z2 * 4);
    const uint32_t sstride = (uint32_t)a.M * Z2 * 4u;
    float kl = 0.f;
    float la[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // LA: L <= 8 on this path
    for (int j = lane; j < Z; j += 64) {
        const uint32_t o = ((uint32_t)m * Z2 + j) * 4u;
        const float mu = slab_sum(bsl, o, sstride, a.nslab, true, a.b4[j]);
        const float lv = slab_sum(bsl, o + Z * 4u, sstride, a.nslab, true, a.b5[j]);
        a.mu[(int64_t)m * Z + j] = mu;
        a.lv[(int64_t)m * Z + j] = lv;
        const float sd = fexp(0.5f * lv);
        kl += 0.5f * (1.f + lv - mu * mu - fexp(lv));
        for (int l = 0; l < a.L; ++l) {
            float e = 0.f;
            if (a.mode != MODE_RECON) {
                if (a.eps_mode == 0) e = philox_normal(a.seed, (uint32_t)grow, (uint32_t)(l * Z + j), c23);
                else e = a.eps_in[((int64_t)l * a.eps_in_ld + m) * Z + j];
            }
            const float z = mu + sd * e;
            const int64_t o = ((int64_t)l * a.M + m) * Z + j;
            a.eps[o] = e;
            a.z[o] = (bf16_t)f2bf(z);
            if (a.est == EST_LA && l < 8) {
                // log p(z) - log q(z|x) = -z^2/2 + lv/2 + (z - mu)^2 e^{-lv} / 2
                la[l] += -0.5f * z * z + 0.5f * lv + 0.5f * e * e;
            }
        }
    }
    if (a.est == EST_LA) {
        for (int l = 0; l < a.L && l < 8; ++l) {
            float v = la[l];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) a.kl_part[(int64_t)l * a.M + m] = v;
        }
    } else {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) kl += __shfl_xor(kl, o, 64);
        if (lane == 0) a.kl_part[m] = kl;
    }
}

// [dMu | dLv] from the dZ slabs (LA direct terms folded as in the
// fp32 path), stored bf16 for the dh / dW45 GEMMs; column sums per 16-row block for the
// b4 / b5 gradients.  Grid (row blocks of 16, column blocks of 64); wave w owns rows
// 4w..4w+3 of the block and lane = one of 64 consecutive columns of [dMu | dLv]
// (coalesced along the latent index); the 4 rows' loads are independent (unrolled), and
// the 4 waves' column sums are combined in fixed order.
constexpr int kLbRows = 16;
__global__ __launch_bounds__(256) void latent_bwd_kernel(LatentArgs a) {
    __shared__ float red[4][64];
    const int Z = a.Z, Z2 = 2 * Z;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y * 64 + lane;
    const int LMZ = a.L * a.M * Z;
    const float sl = a.sc / (float)a.L;
    const bool isv = c >= Z;
    const int j = isv ? c - Z : c;
    const bool cok = c < Z2;
    const rsrc_t bdz = mkbuf(a.dz_slab, (int64_t)a.ndz * LMZ * 4);
    const rsrc_t bmu = mkbuf(a.mu, (int64_t)a.M * Z * 4), blv = mkbuf(a.lv, (int64_t)a.M * Z * 4);
    const rsrc_t bep = mkbuf(a.eps, (int64_t)LMZ * 4);
    int mr[4];
    bool ok[4];
    float mu[4], lv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        mr[r] = blockIdx.x * kLbRows + 4 * w + r;
        ok[r] = cok && mr[r] < a.M;
        const uint32_t o = ok[r] ? (uint32_t)(mr[r] * Z + j) * 4u : kOOB;
        mu[r] = bld(bmu, o);
        lv[r] = bld(blv, o);
    }
    float g[4] = {0.f, 0.f, 0.f, 0.f}, t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int l = 0; l < a.L; ++l) {
        float dz[4], e[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t ol = (uint32_t)((l * a.M + mr[r]) * Z + j) * 4u;
            e[r] = bld(bep, ok[r] ? ol : kOOB);
            dz[r] = 0.f;
        }
        // the four rows' slab loads go out together, 8 slabs per round trip
        for (int s0 = 0; s0 < a.ndz; s0 += 8) {
            float v[4][8];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t ol = (uint32_t)(((s0 + u) * a.L * a.M + l * a.M + mr[r]) * Z + j) * 4u;
                    v[r][u] = bld(bdz, (ok[r] && s0 + u < a.ndz) ? ol : kOOB);
                }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int u = 0; u < 8; ++u) dz[r] += v[r][u];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float sd = fexp(0.5f * lv[r]);
            const float z = mu[r] + sd * e[r];
            if (!isv) {
                g[r] += dz[r];
                if (a.est == EST_LA) t[r] += -z;
            } else {
                g[r] += dz[r] * 0.5f * sd * e[r];
                if (a.est == EST_LA) t[r] += 0.5f - 0.5f * z * sd * e[r];
            }
        }
    }
    float cs = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float v;
        if (a.est == EST_LA) v = g[r] + sl * t[r];
        else v = isv ? g[r] + a.sc * 0.5f * (1.f - fexp(lv[r])) : g[r] - a.sc * mu[r];
        if (ok[r]) {
            a.dmulv[(int64_t)mr[r] * Z2 + c] = (bf16_t)f2bf(v);
            cs += v;
        }
    }
    red[w][lane] = cs;
    __syncthreads();
    if (w == 0 && cok)
        a.colpart[(int64_t)blockIdx.x * Z2 + c] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// ---------------------------------------------------------------- 16-byte forms
// The two latent kernels above move ~50 MB each at config 5 (B = 8192, Z = 128): the
// split-K slabs dominate.  With one 4-byte element per lane they ran at 2-3 TB/s; these
// forms (Z % 4 == 0, 16-B aligned operands; the host checks) give each lane four
// consecutive latent columns, so every slab / mu / lv / eps access is one 16-byte load, and
// latent_bwd_v4 owns BOTH outputs of a latent index (dMu at column j, dLv at Z + j), so
// each dZ slab element is read once instead of twice.  Same arithmetic, same slab order.
DEV void st_bf16x4(bf16_t* p, f32x4 v) {
    const uint32_t lo = f2bf2(v[0], v[1]), hi = f2bf2(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}

// Fixed-order sum of n slab float4s (8 loads per round trip), added to init.
DEV f32x4 slab_sum4(rsrc_t b, uint32_t off, uint32_t stride, int n, bool ok, f32x4 init) {
    f32x4 acc = init;
    for (int s0 = 0; s0 < n; s0 += 8) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = bld4(b, (ok && s0 + u < n) ? off + (uint32_t)(s0 + u) * stride : kOOB);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    return acc;
}

// latent_fwd_kernel, 16-byte form: a wave owns two rows (lanes 0-31, 32-63), a lane four
// latent columns per pass (j0 = 4 lane', + 128 per pass).  Grid ceil(M / 8), 256 threads.
__global__ __launch_bounds__(256) void latent_fwd_v4_kernel(LatentArgs a) {
    const int lane = threadIdx.x & 63, hl = lane & 31;
    const int m = blockIdx.x * 8 + (threadIdx.x >> 5);
    const bool rok = m < a.M;
    const int Z = a.Z, Z2 = 2 * Z;
    const int64_t brow = a.rows.order ? (int64_t)a.rows.order[*a.rows.cursor] : 0;
    const int64_t grow = brow * a.row_base_mul + a.row_base_add + m;
    const uint64_t c23 = philox_c23(*a.step, a.domain);
    const rsrc_t bsl = mkbuf(a.ml_slab, (int64_t)a.nslab * a.M * Z2 * 4);
    const rsrc_t bb4 = mkbuf(a.b4, (int64_t)Z * 4), bb5 = mkbuf(a.b5, (int64_t)Z * 4);
    const uint32_t sstride = (uint32_t)a.M * Z2 * 4u;
    float kl = 0.f;
    float la[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // LA: L <= 8 on this path
    for (int j = 4 * hl; j < Z; j += 128) {
        const bool ok = rok;
        const uint32_t o = ((uint32_t)m * Z2 + j) * 4u;
        const f32x4 b4v = bld4(bb4, (uint32_t)j * 4u), b5v = bld4(bb5, (uint32_t)j * 4u);
        const f32x4 mu = slab_sum4(bsl, o, sstride, a.nslab, ok, b4v);
        const f32x4 lv = slab_sum4(bsl, o + Z * 4u, sstride, a.nslab, ok, b5v);
        if (!ok) continue;
        *reinterpret_cast<f32x4*>(a.mu + (int64_t)m * Z + j) = mu;
        *reinterpret_cast<f32x4*>(a.lv + (int64_t)m * Z + j) = lv;
        f32x4 sd;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            sd[k] = fexp(0.5f * lv[k]);
            kl += 0.5f * (1.f + lv[k] - mu[k] * mu[k] - fexp(lv[k]));
        }
        for (int l = 0; l < a.L; ++l) {
            f32x4 e = zero4();
            if (a.mode != MODE_RECON) {
                if (a.eps_mode == 0) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) e[k] = philox_normal(a.seed, (uint32_t)grow, (uint32_t)(l * Z + j + k), c23);
                } else {
                    e = *reinterpret_cast<const f32x4*>(a.eps_in + ((int64_t)l * a.eps_in_ld + m) * Z + j);
                }
            }
            f32x4 z;
#pragma unroll
            for (int k = 0; k < 4; ++k) z[k] = mu[k] + sd[k] * e[k];
            const int64_t oz = ((int64_t)l * a.M + m) * Z + j;
            *reinterpret_cast<f32x4*>(a.eps + oz) = e;
            st_bf16x4(a.z + oz, z);
            if (a.est == EST_LA && l < 8) {
#pragma unroll
                for (int k = 0; k < 4; ++k) la[l] += -0.5f * z[k] * z[k] + 0.5f * lv[k] + 0.5f * e[k] * e[k];
            }
        }
    }
    // row sums over the 32 lanes of the half-wave
    if (a.est == EST_LA) {
        for (int l = 0; l < a.L && l < 8; ++l) {
            float v = la[l];
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (hl == 0 && rok) a.kl_part[(int64_t)l * a.M + m] = v;
        }
    } else {
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) kl += __shfl_xor(kl, o, 64);
        if (hl == 0 && rok) a.kl_part[m] = kl;
    }
}

// latent_bwd_kernel, 16-byte form: block (16-row block, 128 latent columns), 256 threads =
// 8 row slots x 32 lanes of 4 columns; a thread owns rows rs and rs + 8 and BOTH outputs of
// its columns.  Column partials for b4 / b5: per row slot (rows rs + rs + 8), then the 8
// slots in order.
__global__ __launch_bounds__(256) void latent_bwd_v4_kernel(LatentArgs a) {
    __shared__ float red[8][256];
    const int Z = a.Z, Z2 = 2 * Z;
    const int rs = threadIdx.x >> 5, cl = threadIdx.x & 31;
    const int j = blockIdx.y * 128 + 4 * cl;
    const bool jok = j < Z;
    const int LMZ = a.L * a.M * Z;
    const float sl = a.sc / (float)a.L;
    const rsrc_t bdz = mkbuf(a.dz_slab, (int64_t)a.ndz * LMZ * 4);
    const rsrc_t bmu = mkbuf(a.mu, (int64_t)a.M * Z * 4), blv = mkbuf(a.lv, (int64_t)a.M * Z * 4);
    const rsrc_t bep = mkbuf(a.eps, (int64_t)LMZ * 4);
    int mr[2];
    bool ok[2];
    f32x4 mu[2], lv[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        mr[r] = blockIdx.x * kLbRows + rs + 8 * r;
        ok[r] = jok && mr[r] < a.M;
        const uint32_t o = ok[r] ? (uint32_t)(mr[r] * Z + j) * 4u : kOOB;
        mu[r] = bld4(bmu, o);
        lv[r] = bld4(blv, o);
    }
    f32x4 g[2] = {zero4(), zero4()}, gv[2] = {zero4(), zero4()}, tm[2] = {zero4(), zero4()}, tv[2] = {zero4(), zero4()};
    for (int l = 0; l < a.L; ++l) {
        f32x4 e[2], dz[2];
        const uint32_t sstride = (uint32_t)LMZ * 4u;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const uint32_t ol = (uint32_t)((l * a.M + mr[r]) * Z + j) * 4u;
            e[r] = bld4(bep, ok[r] ? ol : kOOB);
            dz[r] = zero4();
        }
        // both rows' slab loads together, 8 slabs per round trip
        for (int s0 = 0; s0 < a.ndz; s0 += 8) {
            f32x4 v[2][8];
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t ol = (uint32_t)((l * a.M + mr[r]) * Z + j) * 4u + (uint32_t)(s0 + u) * sstride;
                    v[r][u] = bld4(bdz, (ok[r] && s0 + u < a.ndz) ? ol : kOOB);
                }
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int u = 0; u < 8; ++u) dz[r] += v[r][u];
        }
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float sd = fexp(0.5f * lv[r][k]);
                const float z = mu[r][k] + sd * e[r][k];
                g[r][k] += dz[r][k];
                gv[r][k] += dz[r][k] * 0.5f * sd * e[r][k];
                if (a.est == EST_LA) {
                    tm[r][k] += -z;
                    tv[r][k] += 0.5f - 0.5f * z * sd * e[r][k];
                }
            }
    }
    f32x4 cm = zero4(), cv = zero4();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        f32x4 dm, dl;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (a.est == EST_LA) {
                dm[k] = g[r][k] + sl * tm[r][k];
                dl[k] = gv[r][k] + sl * tv[r][k];
            } else {
                dm[k] = g[r][k] - a.sc * mu[r][k];
                dl[k] = gv[r][k] + a.sc * 0.5f * (1.f - fexp(lv[r][k]));
            }
        }
        if (ok[r]) {
            st_bf16x4(a.dmulv + (int64_t)mr[r] * Z2 + j, dm);
            st_bf16x4(a.dmulv + (int64_t)mr[r] * Z2 + Z + j, dl);
            cm += dm;
            cv += dl;
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        red[rs][4 * cl + k] = cm[k];
        red[rs][128 + 4 * cl + k] = cv[k];
    }
    __syncthreads();
    const int t = threadIdx.x;
    const int jc = blockIdx.y * 128 + (t & 127);
    if (jc < Z) {
        float s = red[0][t];
#pragma unroll
        for (int q = 1; q < 8; ++q) s += red[q][t];
        a.colpart[(int64_t)blockIdx.x * Z2 + (t < 128 ? jc : Z + jc)] = s;
    }
}

// Split-K weight gradients: sum the slabs in fixed order, then the optimizer rule.
struct WReduceArgs {
    const float* slab; int nslab; int M, N;   // slabs [nslab][M][N]
    ColMap map; Opt opt; bf16_t* shadow;      // shadow: this weight's GEMM-layout copy
};
__global__ __launch_bounds__(256) void wreduce_opt_kernel(WReduceArgs w) {
    const int64_t MN = (int64_t)w.M * w.N;
    const int64_t stride = (int64_t)gridDim.x * 256;
    const rsrc_t bs = mkbuf(w.slab, (int64_t)w.nslab * MN * 4);
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < MN; e += stride) {
        const float g = slab_sum(bs, (uint32_t)e * 4u, (uint32_t)MN * 4u, w.nslab, true, 0.f);
        const int m = (int)(e / w.N), n = (int)(e % w.N);
        w.opt.apply(w.map.at(m, n), e, g);
    }
}

// ELBO partials, stage 1: block b sums a contiguous chunk of the per-row log p and
// KL / LA partials in fp64 (fixed order) -> parts[2b], parts[2b + 1].
constexpr int kElboBlocks = 256;
__global__ __launch_bounds__(256) void elbo_partial_kernel(ElboArgs e, double* parts) {
    __shared__ double sh[256];
    const int64_t clp = (e.n_lp + gridDim.x - 1) / gridDim.x, ckl = (e.n_kl + gridDim.x - 1) / gridDim.x;
    const int64_t lp0 = blockIdx.x * clp, lp1 = min(e.n_lp, lp0 + clp);
    const int64_t kl0 = blockIdx.x * ckl, kl1 = min(e.n_kl, kl0 + ckl);
    double lp = 0, kl = 0;
    // 8 loads per round trip (buffer range check zero-fills the tail), fixed order
    const rsrc_t blp = mkbuf(e.lp_part, e.n_lp * 4), bkl = mkbuf(e.kl_part, e.n_kl * 4);
    for (int64_t i0 = lp0 + threadIdx.x; i0 < lp1; i0 += 8 * 256) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = bld(blp, i0 + u * 256 < lp1 ? (uint32_t)(i0 + u * 256) * 4u : kOOB);
#pragma unroll
        for (int u = 0; u < 8; ++u) lp += v[u];
    }
    for (int64_t i0 = kl0 + threadIdx.x; i0 < kl1; i0 += 8 * 256) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = bld(bkl, i0 + u * 256 < kl1 ? (uint32_t)(i0 + u * 256) * 4u : kOOB);
#pragma unroll
        for (int u = 0; u < 8; ++u) kl += v[u];
    }
    lp = block_sum256(lp, sh);
    kl = block_sum256(kl, sh);
    if (threadIdx.x == 0) { parts[2 * blockIdx.x] = lp; parts[2 * blockIdx.x + 1] = kl; }
}

// ELBO stage 2 (one workgroup): the stage-1 sums in fixed order, then the step outputs.
DEV void elbo_finish(const ElboArgs& e, const double* parts, int n) {
    __shared__ double sh[256];
    double lp = 0, kl = 0;
    for (int i = threadIdx.x; i < n; i += 256) { lp += parts[2 * i]; kl += parts[2 * i + 1]; }
    lp = block_sum256(lp, sh);
    kl = block_sum256(kl, sh);
    if (threadIdx.x == 0) elbo_emit(e, lp, kl, 0.0);
}
__global__ __launch_bounds__(256) void elbo_final_kernel(ElboArgs e, const double* parts, int n) {
    elbo_finish(e, parts, n);
}

// Bias gradients from the epilogues' column partials (fixed order), optimizer rule, and
// one extra workgroup that finishes the ELBO and advances cursor / step.  A block owns
// 64 consecutive bias columns; its 4 waves split the partial rows (lane = column) with
// 8 loads in flight each, then wave 0 sums the 4 wave totals in order.
struct BiasSeg {
    const float* part; int nrb; int N;   // partials [nrb][N]
    ColMap map;                           // column -> arena index (biases: ld = 0)
};
struct BiasArgs {
    BiasSeg seg[4]; int nseg;
    int segblk[4];                        // blocks per segment: ceil(N / 64)
    int total;                            // sum of the segments' N
    Opt opt;
    ElboArgs elbo;
    const double* elbo_parts; int n_elbo_parts;
};
__global__ __launch_bounds__(256) void bias_opt_kernel(BiasArgs b) {
    if (blockIdx.x == gridDim.x - 1) {
        elbo_finish(b.elbo, b.elbo_parts, b.n_elbo_parts);
        return;
    }
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // blocks never straddle segments (segblk: ceil(N / 64) blocks per segment), so the
    // segment and its partials' buffer descriptor are block-uniform
    int bid = blockIdx.x, s = 0;
    while (s < b.nseg - 1 && bid >= b.segblk[s]) { bid -= b.segblk[s]; ++s; }
    const BiasSeg& g = b.seg[s];
    const int e = bid * 64 + lane;
    const bool ok = e < g.N;
    // 32 loads in flight per round trip (one round at 128 partial rows), accumulated into 8
    // running sums: row w + 4k + 32i goes to sum k in increasing i
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const rsrc_t bp = mkbuf(g.part, (int64_t)g.nrb * g.N * 4);
    for (int r0 = w; r0 < g.nrb; r0 += 128) {
        float v[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const int r = r0 + 4 * u;
            v[u] = bld(bp, (ok && r < g.nrb) ? (uint32_t)((int64_t)r * g.N + e) * 4u : kOOB);
        }
#pragma unroll
        for (int u = 0; u < 32; ++u) acc[u & 7] += v[u];
    }
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) v += acc[u];
    red[w][lane] = v;
    __syncthreads();
    if (w == 0 && ok) {
        const float t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
        b.opt.apply(g.map.at(0, e), -1, t);
    }
}

// DP: after the all-reduce of [grad arena | SGVB], the replicated optimizer over the
// whole arena, rewriting the bf16 shadow.
__global__ __launch_bounds__(256) void adagrad_bf16_kernel(Opt o, int64_t P, DpRange r, ShadowMap m, ElboArgs e) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t n = r.total();
    const rsrc_t bti = mkbuf(o.th_in, P * 4), bto = mkbuf(o.th_out, P * 4);
    const rsrc_t bac = mkbuf(o.accum, P * 4), bgr = mkbuf(o.grad, P * 4);
    // U grid-stride elements per memory round trip (loads before stores), the rule of
    // Opt::apply, then theta' and its bf16 shadow copy
    constexpr int U = 8;
    for (int64_t v0 = (int64_t)blockIdx.x * 256 + threadIdx.x; v0 < n; v0 += U * stride) {
        uint32_t off[U];
        float th[U], ac[U], gr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t v = v0 + u * stride;
            off[u] = v < n ? (uint32_t)r.at(v) * 4u : kOOB;
            th[u] = bld(bti, off[u]);
            ac[u] = bld(bac, off[u]);
            gr[u] = bld(bgr, off[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (off[u] == kOOB) continue;
            const int64_t i = off[u] >> 2;
            const float gg = gr[u] - o.prior * th[u];
            const float a = ac[u] + gg * gg;
            const float tn = th[u] + o.lr * gg / (__builtin_amdgcn_sqrtf(a) + o.eps) - o.decay * th[u] * th[u];
            bst(bac, off[u], a);
            bst(bto, off[u], tn);
            const int64_t si = m.at(i);
            if (si >= 0) o.shadow_out[si] = (bf16_t)f2bf(tn);
        }
    }
    if (r.book && blockIdx.x == 0 && threadIdx.x == 0) {
        const double v = (double)o.grad[P] * e.inv_bglob;
        elbo_store(e, (float)v);
        e.epoch[0] += v;
        e.epoch[1] += 1.0;
        if (e.cursor) advance_cursor(e.cursor);
        *e.step += 1;
    }
}

}  // namespace VAEB_H16NS
}  // namespace vaeb
