// kernels_aux.hpp -- the weight-gradient / optimizer end of the SGVB step and the
// reductions (/root/reference/VAEB.py:385-444).
#pragma once
#include "fused.hpp"

namespace vaeb {

// ----------------------------------------------------------------- ELBO reduction
// The context's 64-bit control block (vaeb_hip.hip vaeb_create): slots 0, 1 the epoch ELBO
// accumulators (double), 2 the sticky step status, 3 the last step's SGVB / B (float), 4
// the fixed-point hand-off range-guard word, then the hand-off accumulators (latent.hpp).
constexpr int kBlkStatus = 2, kBlkElbo = 3, kBlkFxErr = 4, kBlkAcc = 5;

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

DEV void elbo_emit(const ElboArgs& e, double lp, double kl, double fv);

// Fixed-order strided sum of p[0, n) for one 256-thread workgroup: thread t adds
// p[t], p[t + 256], ... in index order; U of its loads are in flight per round trip
// (a load -> add chain per element cost one memory latency each: 22 of them over the
// MNIST log p partials, 9 us for the FV step's ELBO launch).
template <int U>
DEV double strided_sum(const float* p, int64_t n) {
    const rsrc_t b = mkbuf(p, n * 4);
    double s = 0;
    for (int64_t i0 = threadIdx.x; i0 < n; i0 += 256 * U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + (int64_t)u * 256;
            v[u] = bld(b, i < n ? (uint32_t)(i * 4) : kOOB);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) s += (double)v[u];
    }
    return s;
}

DEV double wave_sum64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Fixed-order workgroup sum for 256 threads: a butterfly per wave, then the wave sums in
// order (one barrier instead of block_sum256's eight).  Valid on thread 0.
DEV double block_sum256w(double v, double* sh) {
    v = wave_sum64(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    return ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

// Deterministic (fixed-order) reduction by one 256-thread workgroup: strided per-thread
// sums, a butterfly within each wave, then the four wave sums in wave order.
// cursor += 1 and next = order[cursor] (tile_engine.hpp, kCtlNext)
DEV void advance_cursor(int* cursor) {
    const int c1 = *cursor + 1;
    *cursor = c1;
    cursor[kCtlNext] = cursor[kCtlOrder + c1];
}

DEV void elbo_reduce(const ElboArgs& e, double* sh) {
    double v[3] = {strided_sum<16>(e.lp_part, e.n_lp), strided_sum<4>(e.kl_part, e.n_kl),
                   strided_sum<4>(e.fv_part, e.n_fv)};
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        v[k] = wave_sum64(v[k]);
        if (lane == 0) sh[wave * 3 + k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double r[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) r[k] = ((sh[k] + sh[3 + k]) + sh[6 + k]) + sh[9 + k];
    elbo_emit(e, r[0], r[1], r[2]);
}

// The step's [SGVB / B, flags] into the context's mapped host slot (vaeb_hip.hip
// vaeb_update) as ONE 8-byte store, so the host that polls the flags word (2 = written,
// | 1 = the sticky status is set) reads the value of the same store.
DEV void elbo_store(const ElboArgs& e, float v) {
    const unsigned long long st = reinterpret_cast<const unsigned long long*>(e.epoch)[kBlkStatus];
    const unsigned long long w =
        (unsigned long long)__builtin_bit_cast(uint32_t, v) | ((unsigned long long)(st ? 3u : 2u) << 32);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(e.elbo_out), w, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// The step's scalar outputs from the reduced sums (thread 0 of the reducing workgroup).
DEV void elbo_emit(const ElboArgs& e, double lp, double kl, double fv) {
    // LB: sum logp / L + sum KL (VAEB.py:339-344); LA: (sum logp + sum(prior-logQ)) / L
    // (VAEB.py:327-328); FV: B * (sum logp + sum KL) + thetaPrior (VAEB.py:364).
    const double data = (e.est == EST_LA) ? (lp + kl) / e.L : lp / e.L + kl;
    const double sg = (e.est == EST_FV) ? e.data_mul * data + fv : data;
    if (e.epoch) {
        // training step: fold the fixed-point hand-offs' range-guard word (latent.hpp fx_inc,
        // slot 4 of the control block) into the sticky status slot 2 the host reads at its
        // next sync (vaeb_update / vaeb_epoch_elbo -> VAEB_ERR_NUMERIC); cleared for the next step
        unsigned long long* w = reinterpret_cast<unsigned long long*>(e.epoch);
        const unsigned long long err =
            __hip_atomic_exchange((__attribute__((address_space(1))) unsigned long long*)(w + kBlkFxErr), 0ull,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (err) w[kBlkStatus] |= err;
    }
    if (e.eval_acc) { e.eval_acc[0] += data; e.eval_acc[1] = fv; }
    if (e.dp_slot) {
        *e.dp_slot = (float)sg;
    } else if (e.elbo_out) {
        const double v = sg * e.inv_bglob;
        elbo_store(e, (float)v);
        e.epoch[0] += v;
        e.epoch[1] += 1.0;
    }
    if (e.cursor) advance_cursor(e.cursor);
    if (e.step) *e.step += 1;
}

// A short batch order as a kernel argument (vaeb_hip.hip upload_order): writes
// [cursor = 0, cur_batch = 0, next = order[0], order...] on the step stream.
constexpr int kArgOrder = 960;   // 3.8 KB of kernel argument
struct OrderArg { int n; int v[kArgOrder]; };
__global__ __launch_bounds__(256) void set_order_kernel(int* ictl, OrderArg u) {
    for (int i = threadIdx.x; i < u.n; i += 256) ictl[kCtlOrder + i] = u.v[i];
    if (threadIdx.x == 0) {
        ictl[0] = 0;
        ictl[1] = 0;
        ictl[kCtlNext] = u.n > 0 ? u.v[0] : 0;
    }
}

// Measurement helper: holds the stream for ~`ticks` x 10 ns (s_memrealtime runs at
// 100 MHz) so that the host can enqueue a whole eager step behind it; the events
// between the step's launches then time back-to-back kernels, as in a graph replay.
__global__ __launch_bounds__(64) void delay_kernel(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// Diagnostics: every CU busy with MFMA work for `us` microseconds (s_memrealtime at 100 MHz),
// result kept live through a store that never happens (a < 0 never holds).
__global__ __launch_bounds__(256) void busy_kernel(uint64_t ticks, float* sink) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    float a = (float)(threadIdx.x & 7) * 1e-3f, b = 1e-3f;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
#pragma unroll
        for (int i = 0; i < 32; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
    if (acc[0] < -1.f) sink[threadIdx.x] = acc[1];
}

// Posterior-sample reconstruction (VAEB.py:277-291): acc = acc + y in sample order
// (first sample: acc = y), and on the last sample acc /= n_samples.
__global__ __launch_bounds__(256) void recon_accum_kernel(float* acc, const float* y, int64_t n, int first,
                                                          float scale) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        float v = first ? y[i] : acc[i] + y[i];
        acc[i] = scale != 0.f ? v / scale : v;
    }
}

__global__ __launch_bounds__(256) void elbo_kernel(ElboArgs e) {
    __shared__ double sh[256];
    elbo_reduce(e, sh);
}

// ----------------------------------------------------------------- optimizer rule
// Parameters ping-pong between two arenas: a step reads theta_in (every phase of the
// step sees the pre-update values, as Theano's simultaneous updates do, VAEB.py:438-442)
// and writes theta_out, so the optimizer of one weight group can run while later phases
// of the same step still read the old weights.  Accumulators are updated in place (only
// the owning element reads them).
struct OptArgs {
    const float* theta_in; float* theta_out; float* acc; float* grad;
    float lr, eps, prior, decay;  // decay = lr*eps for the mean_map variant, else 0
    int update, store_grad;
};

// VAEB.getUpdates (VAEB.py:438-442) on one element, prior folded in (VAEB.py:389-390):
//   g = dSGVB/dtheta - prior*theta;  acc += g^2;  theta += lr*g/(sqrt(acc)+eps) [- decay*theta^2]
DEV float opt_rule(const OptArgs& o, float th, float& acc, float dsg) {
    const float g = dsg - o.prior * th;
    acc += g * g;
    // hardware sqrt / reciprocal (1 ulp each) instead of the IEEE-exact expansions: a
    // weight-gradient epilogue wave ran ~50 instructions per parameter on them
    return th + o.lr * g * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(acc) + o.eps) - o.decay * th * th;
}

// ----------------------------------------------------------------- weight gradients
// C[i][j] = sum_k At[k][i] * B[k][j] over the minibatch rows k (K padded to 16; pad rows
// of every delta are zero), i = weight row, with row i == rowsW the all-ones row so the
// bias gradient (the column sum of the delta) is computed by the same MFMAs.  B is the
// column concatenation of up to two delta arrays (dA2 | dA6 -> W2 | W6, dMu | dLv ->
// W4 | W5).  A 256-thread workgroup owns a 64 x 64 tile: both operand panels are staged
// through LDS with 16-byte loads (K rows x 64 floats, pitch 68 to spread the column
// reads over the banks), then wave w computes rows 16w..16w+15 x 64 columns
// (4 accumulators sharing one A fragment).  The epilogue applies prior + Adagrad
// (theta / acc prefetched before the panels) or stores the gradient (DP / introspection).
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
constexpr bool kNoTV = false;
constexpr int kWT = 64;   // weight rows (i) per tile; the columns per tile are 16 * TS (wgrad_body)
constexpr int kWKB = 128;
constexpr int kWP = 68;

struct WGroup {
    const float* at; int ld_at; int klim_at; int at_is_x;
    int rowsW;
    const float* b0; int ld0; int N0;
    const float* b1; int ld1; int N1;
    int K;
    int64_t offW0, offb0, offW1, offb1;
    int tiles_j, wg_begin, wg_end;
};

// dA3 = ([dMu | dLv] [W4 | W5]^T) (1 - h^2) computed inside the dW3 workgroups (the
// folded latent backward, latent_bwd.hpp): the B panel of dW3 = [X | 1]^T dA3 is formed
// from dMuLv, W4 / W5 (pre-update arena) and h instead of being loaded.
// Deferred latent backward (VAEB_BWD_DEFER, default where the slab form is chosen: fan-in >
// 16).  The dhd tiles of the previous launch stored their partial dZ slabs with plain stores
// and ended (the kernel boundary publishes them: no drain, no ticket in that launch); here
// `nred` reducer workgroups -- dispatched right after the ELBO one -- each sum one (row block,
// latent column group) of the slabs in fixed order, form [dMu | dLv] and publish it
// write-through (sc1), every storing wave drained, behind ONE agent-scope add per workgroup
// on one counter.  The consumers (the dW3 workgroups' dA3 panel and the dW4 | dW5 group)
// poll that counter with sc1 loads from one lane, join a workgroup barrier and read [dMu |
// dLv] with sc1 loads only: MI355X_MICROARCH.md's hand-off table row 1, the four conditions
// latent.hpp arrive_last cites.  The counter is zeroed by the dhd launch (a plain store the
// boundary publishes).  The poll is bounded: a timeout sets the guard word (reported as a
// step status) instead of hanging the GPU.
struct LatRed {
    const float* slab;                 // [L][nrb][nctH][Z][16] partial dZ slabs
    const float *mu, *lv, *eps, *z;    // [Mbp][Z]; [L][Mbp][Z]
    float* dZ;                         // [L][Mbp][Z] (kept for inspection, as the ticketed form)
    float* dml;                        // [Mbp][2Z] [dMu | dLv]: the handed-off bytes
    int* cnt;                          // completion counter, kLatCnt replicas kLatCntStride apart
    uint64_t* guard;                   // blk[kBlkFxErr]: timeout bit
    int nred, ngrp, zg, nctH, L, est, Mb, Mbp, Z;
    float sc;
};
// The completion counter can be kept in kLatCnt replicas on lines of their own (MI355X_MICROARCH.md's
// hand-off table, row 2; -DVAEB_LAT_CNT=8 build): each reducer adds to every replica with ONE
// wave instruction of kLatCnt lanes, and a consumer polls the replica of its round-robin slot
// (blockIdx.x % 8), so the launch's 448 pollers spread over 8 lines.  Round 4 A/B (alternating
// 4000-step runs): with 16-byte publication stores (-DVAEB_LAT_ST4) 34.51 / 34.53 µs, the single
// counter with those stores 35.06 / 35.17, the single counter with dword stores (the default)
// 34.51 / 34.35; the timeline build saw the poll return ~2 µs earlier with replicas, the
// production step did not.  Eight copies of [dMu | dLv] as well (one per XCD): 10.86 vs 10.57 µs.
constexpr int kLatCnt = 1, kLatCntStride = 16;   // replicas 64 B apart
DEV int lat_slot() { return (int)(blockIdx.x & (kLatCnt - 1)); }
struct Da3Src {
    const float *dml, *W4, *W5, *h;
    float* dA3;           // the column slice is also stored (by the D-row tile 0 workgroups)
    int Z, H, Mb, Mbp;
    LatRed red;           // red.nred > 0: [dMu | dLv] is produced in this launch (deferred form)
};
constexpr uint64_t kGuardHandoffTimeout = 4;

// One reducer workgroup (256 threads): row block rb, latent columns [j0, j0 + nj).  Element
// thread t < 16 nj owns (row rb * 16 + t / nj, column j0 + t % nj).
// dbg (timeline build): stamp slots of this reducer (5 slab loads landed, 2 [dMu | dLv] formed,
// 6 stores drained)
DEV void lat_reduce_wg(const LatRed& r, int wi, f32x4* red, float (*dzs)[17], uint64_t* dbg = nullptr) {
    const int Z = r.Z, nrb = r.Mbp >> 4;
    const int rb = wi / r.ngrp, cg = wi - rb * r.ngrp;
    const int j0 = cg * r.zg, nj = min(r.zg, Z - j0);
    const int nf = 4 * nj, np = 256 / nf;   // float4 per slab group (column, row quad); partitions
    const int t = threadIdx.x, f = t % nf, part = t / nf;
    const bool el = t < 16 * nj;
    const int ml = el ? t / nj : 0, jj = el ? t - (t / nj) * nj : 0;
    const int m = rb * 16 + ml, j = j0 + jj;
    const bool valid = el && m < r.Mb;
    // the element's own operands ride the round trip of the first slab loads
    const uint32_t oj = valid ? (uint32_t)(m * Z + j) * 4u : kOOB;
    const float mu = bld(mkbuf(r.mu, (int64_t)r.Mbp * Z * 4), oj);
    const float lv = bld(mkbuf(r.lv, (int64_t)r.Mbp * Z * 4), oj);
    float epre[kLP], zpre[kLP];
    const rsrc_t be = mkbuf(r.eps, (int64_t)r.L * r.Mbp * Z * 4), bz = mkbuf(r.z, (int64_t)r.L * r.Mbp * Z * 4);
#pragma unroll
    for (int l = 0; l < kLP; ++l) {
        const uint32_t o = (valid && l < r.L) ? (uint32_t)((l * r.Mbp + m) * Z + j) * 4u : kOOB;
        epre[l] = bld(be, o);
        zpre[l] = r.est == EST_LA ? bld(bz, o) : 0.f;
    }
    const rsrc_t bs = mkbuf(r.slab, (int64_t)r.L * r.Mbp * r.nctH * Z * 4);
    float dzsum = 0.f, dzes = 0.f;
    for (int l = 0; l < r.L; ++l) {
        const int64_t first = (int64_t)(l * nrb + rb) * r.nctH;
        constexpr int SV = 8;
        f32x4 sum = zero4();
        for (int c0 = part; c0 < r.nctH; c0 += SV * np) {
            f32x4 v[SV];
#pragma unroll
            for (int u = 0; u < SV; ++u) {
                const int ct = c0 + u * np;
                v[u] = bld4(bs, (part < np && ct < r.nctH) ? (uint32_t)((((first + ct) * Z + j0) * 4 + f) * 16) : kOOB);
            }
#pragma unroll
            for (int u = 0; u < SV; ++u) sum += v[u];
        }
        if (VAEB_DBG_ON(dbg) && l == 0 && t == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            dbg[5] = __builtin_amdgcn_s_memrealtime();
        }
        red[t] = sum;
        __syncthreads();
        if (t < nf) {   // the np partition sums in order: deterministic
            f32x4 s4 = red[t];
            for (int pp = 1; pp < np; ++pp) s4 += red[pp * nf + t];
#pragma unroll
            for (int k = 0; k < 4; ++k) dzs[t >> 2][4 * (t & 3) + k] = s4[k];
        }
        __syncthreads();
        const float dz = valid ? dzs[jj][ml] : 0.f;
        const float e = l < kLP ? epre[l] : (valid ? r.eps[((int64_t)l * r.Mbp + m) * Z + j] : 0.f);
        dzsum += dz;
        dzes += dz * e;
        if (el) r.dZ[((int64_t)l * r.Mbp + m) * Z + j] = dz;
        __syncthreads();   // red / dzs are reused by the next plane
    }
    // [dMu | dLv] (VAEB.py:315-346): LB / FV the KL direct terms, LA the
    // prior - logQ direct terms (latent_bwd.hpp latent_bwd_elem)
    const float sl = r.sc / (float)r.L, sd = fexp(0.5f * lv);
    float dmu = 0.f, dlv = 0.f;
    if (valid) {
        if (r.est == EST_LA) {
            float tm = 0.f, tv = 0.f;
            for (int l = 0; l < r.L; ++l) {
                const int64_t ol = ((int64_t)l * r.Mbp + m) * Z + j;
                const float zz = l < kLP ? zpre[l] : r.z[ol];
                const float e = l < kLP ? epre[l] : r.eps[ol];
                tm += -zz;
                tv += 0.5f - 0.5f * zz * sd * e;
            }
            dmu = dzsum + sl * tm;
            dlv = dzes * 0.5f * sd + sl * tv;
        } else {
            dmu = dzsum - r.sc * mu;
            dlv = dzes * 0.5f * sd + r.sc * 0.5f * (1.f - fexp(lv));
        }
    }
    if (VAEB_DBG_ON(dbg) && t == 0) dbg[2] = __builtin_amdgcn_s_memrealtime();
    // publish, write-through (sc1): dword stores (VAEB_LAT_ST4: 16-byte runs staged through LDS);
    // then every storing wave drains, the barrier, one add per counter replica (one instruction)
    const rsrc_t bd = mkbuf(r.dml, (int64_t)r.Mbp * 2 * Z * 4);
    if (false) {
        float* stg = reinterpret_cast<float*>(red);   // [16 rows][2 nj + 1]
        const int sp = 2 * nj + 1;
        __syncthreads();   // (red held the partition sums)
        if (el) {
            stg[ml * sp + jj] = dmu;
            stg[ml * sp + nj + jj] = dlv;
        }
        __syncthreads();
        const int nc4 = nj >> 1;   // 16-byte chunks per row: nj / 4 of dMu, nj / 4 of dLv
        if (t < 16 * nc4) {
            const int row = t / nc4, q = t - row * nc4;
            const int half = q >= (nj >> 2) ? 1 : 0, c4 = q - half * (nj >> 2);
            const int mm = rb * 16 + row;
            f32x4 v;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = stg[row * sp + half * nj + 4 * c4 + k];
            bst4x<16>(bd, (mm < r.Mbp) ? (uint32_t)(mm * 2 * Z + half * Z + j0 + 4 * c4) * 4u : kOOB, v);
        }
    } else if (el) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, dmu), bd, (uint32_t)(m * 2 * Z + j) * 4u, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, dlv), bd, (uint32_t)(m * 2 * Z + Z + j) * 4u, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (VAEB_DBG_ON(dbg) && t == 0) dbg[6] = __builtin_amdgcn_s_memrealtime();
    if (t < kLatCnt)
        __hip_atomic_fetch_add((__attribute__((address_space(1))) int*)(r.cnt + t * kLatCntStride), 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
}

// Consumer side: one lane polls the counter (sc1 loads, s_sleep between polls, bounded), the
// workgroup joins a barrier; every later load of [dMu | dLv] in the workgroup is an sc1 load.
// s_sleep units (64 clocks) between polls: fewer polls of the one counter line (A/B, 4000-step
// runs: 2 -> 34.66 / 34.72 us, 10 -> 34.48 / 34.51, 30 -> 34.34 / 34.35; then 30 -> 34.26 / 34.29,
// 60 -> 34.38 / 34.33, 110 -> 35.61 / 35.55)
constexpr int kPollSleep = 30;
DEV void lat_wait(int* cnt, int nred, uint64_t* const* guard) {
    if (threadIdx.x == 0) {
        typedef __attribute__((address_space(1))) int gi32;
        uint32_t spins = 0;
        while (__hip_atomic_load((gi32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nred) {
            __builtin_amdgcn_s_sleep(kPollSleep);
            if (++spins >= (1u << 20)) {   // ~1 s: never a hang; the step reports a status instead
                __hip_atomic_fetch_or((__attribute__((address_space(1))) unsigned long long*)*guard,
                                      (unsigned long long)kGuardHandoffTimeout, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the sc1 loads below the poll
}

// Kernel arguments of a weight-gradient launch: up to two groups (WGradArgs), or the three
// groups + dA3 source of the folded latent backward's last launch (WGradArgs3).  Separate
// types because the kernarg size shows in every launch that takes it (the 3-group form as
// the common type cost the 2-group launch 6.9 -> 8.6 us).
struct WGradArgs {
    WGroup g[2];
    int ngroups, total_wgs;
    OptArgs opt;
    ElboArgs elbo;
    int with_elbo;
    const float* xbase; const int* cur_batch; int64_t batch_stride;
    int64_t P;
    uint64_t* dbg;
};
// The first 64 bytes of WGradArgs3: every kernel argument a workgroup needs before its first
// operand load (its role, its group, the batch pointer), read as ONE scalar load at entry --
// read field by field, each branch on the previous one cost a dependent scalar round trip
// to the kernarg segment (the deferred reducers' count added one: last launch 10.2 -> 11.4 us).
struct W3Head {
    const float* xbase; const int* cur_batch; int64_t batch_stride;
    int with_elbo, total_wgs, ngroups, nred;   // nred: LatRed reducers ahead of the tiles
    int gb1, gb2;                              // first workgroup of groups 1 and 2
    int* red_cnt;                              // LatRed counter (the consumers' poll)
};
struct WGradArgs3 {
    W3Head hd;
    WGroup g[3];
    OptArgs opt;
    ElboArgs elbo;
    int64_t P;
    uint64_t* dbg;
    Da3Src da3;
};
DEV const float* wa_xbase(const WGradArgs& p) { return p.xbase; }
DEV const int* wa_cur_batch(const WGradArgs& p) { return p.cur_batch; }
DEV int64_t wa_batch_stride(const WGradArgs& p) { return p.batch_stride; }
DEV const float* wa_xbase(const WGradArgs3& p) { return p.hd.xbase; }
DEV const int* wa_cur_batch(const WGradArgs3& p) { return p.hd.cur_batch; }
DEV int64_t wa_batch_stride(const WGradArgs3& p) { return p.hd.batch_stride; }

// [W4 | W5]^T element block B(k, n) = W4[n][k] (k < Z) | W5[n][k - Z] (Z <= k < 2Z), four
// consecutive k at row n (16-byte loads when vz: Z % 4 == 0 and both bases aligned).
DEV f32x4 ld_w45(rsrc_t bw4, rsrc_t bw5, int Z, int H, int n, int k, bool vz) {
    if (vz) return (k < Z) ? kc4(bw4, Z, n, k, H, Z, true) : kc4(bw5, Z, n, k - Z, H, Z, true);
    f32x4 v;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int kk = k + s;
        const bool ok = n < H;
        v[s] = bld(bw4, (ok && kk < Z) ? (uint32_t)(n * Z + kk) * 4u : kOOB) +
               bld(bw5, (ok && kk >= Z && kk < 2 * Z) ? (uint32_t)(n * Z + kk - Z) * 4u : kOOB);
    }
    return v;
}

// dA3 rows [kb, kb + kWKB) x columns [j0, j0 + 16 TS) into the B panel sb (Da3Src): wave
// w of NWV takes the 16-row blocks w, w + NWV, ... (NR = kWKB / 16 / NWV of them); K = 2Z
// <= 64.  Every operand of all NR blocks is issued before the first MFMA (one round trip;
// a per-block load -> MFMA loop cost the launch a second one), the [W4 | W5]^T slice once.
// DEFER (the deferred latent backward, LatRed): [dMu | dLv] is produced in this launch, so its
// loads wait for the reducers' counter and are sc1; the W4 / W5 and h loads go out first.
template <int NWV, int TS, bool DEFER = false>
DEV void da3_panel(const Da3Src& d, int kb, int j0, bool store, float (*sb)[kWP], int* cnt = nullptr, int nred = 0,
                   uint64_t* dbg = nullptr) {   // dbg (timeline build): slot 7 = the poll returned
    constexpr int NR = kWKB / 16 / NWV;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int li = lane & 15, q = lane >> 4;
    const int Z = d.Z, H = d.H, K2 = 2 * d.Z;
    const rsrc_t bd = mkbuf(d.dml, (int64_t)d.Mbp * K2 * 4);
    const rsrc_t bw4 = mkbuf(d.W4, (int64_t)H * Z * 4), bw5 = mkbuf(d.W5, (int64_t)H * Z * 4);
    const rsrc_t bh = mkbuf(d.h, (int64_t)d.Mbp * H * 4);
    const bool vz = (Z & 3) == 0 && aligned16(d.W4) && aligned16(d.W5);
    const bool vd = (K2 & 3) == 0 && aligned16(d.dml);
    const int nkc = (K2 + 15) >> 4;
    f32x4 bw[TS][4], av[NR][4], hv[NR][TS];
#pragma unroll
    for (int ts = 0; ts < TS; ++ts)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            bw[ts][c] = ld_w45(bw4, bw5, Z, c < nkc ? H : 0, j0 + 16 * ts + li, c * 16 + 4 * q, vz);
        }
#pragma unroll
    for (int u = 0; u < NR; ++u) {
        const int r0 = kb + 16 * (wv + NWV * u);
        const int rl = r0 < d.Mbp ? d.Mbp : 0;   // blocks past the padded batch load nothing
        if constexpr (!DEFER)
#pragma unroll
            for (int c = 0; c < 4; ++c) av[u][c] = kc4(bd, K2, r0 + li, c * 16 + 4 * q, c < nkc ? rl : 0, K2, vd);
#pragma unroll
        for (int ts = 0; ts < TS; ++ts) {
            const int n = j0 + 16 * ts + li;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mm = r0 + 4 * q + r;
                hv[u][ts][r] = bld(bh, (n < H && mm < d.Mb) ? (uint32_t)(mm * H + n) * 4u : kOOB);
            }
        }
    }
    if constexpr (DEFER) {
        lat_wait(cnt + lat_slot() * kLatCntStride, nred, &d.red.guard);
        if (VAEB_DBG_ON(dbg) && kb == 0 && threadIdx.x == 0) dbg[7] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int u = 0; u < NR; ++u) {
            const int r0 = kb + 16 * (wv + NWV * u);
            const int rl = r0 < d.Mbp ? d.Mbp : 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                av[u][c] = kc4x<16>(bd, K2, r0 + li, c * 16 + 4 * q, c < nkc ? rl : 0, K2, vd);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < NR; ++u) {
        const int t = wv + NWV * u;
        const int r0 = kb + 16 * t;
        if (r0 >= d.Mbp) break;
#pragma unroll
        for (int ts = 0; ts < TS; ++ts) {
            f32x4 acc = zero4();
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c < nkc) acc = mfma4(av[u][c], bw[ts][c], acc);
            const int n = j0 + 16 * ts + li;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mm = r0 + 4 * q + r;
                const float v = (mm < d.Mb && n < H) ? acc[r] * (1.f - hv[u][ts][r] * hv[u][ts][r]) : 0.f;
                sb[16 * t + 4 * q + r][16 * ts + li] = v;
                if (store && n < H) d.dA3[(int64_t)mm * H + n] = v;
            }
        }
    }
}

// One 64 x (16 TS) tile of group g (passed with a compile-time index, so its fields are
// scalar kernel-argument loads; a dynamic index made hipcc fetch them with serialized
// per-lane vector loads).  NWV = 4 waves (standalone launch) or 8 (a 512-thread fused
// launch): waves w and w + 4 then take alternate K chunks and are summed through LDS.
// DA3: the B panel is dA3, formed in the workgroup (da3_panel) instead of loaded.
// DEFER: the B panel ([dMu | dLv]: dW4 | dW5) or dA3's [dMu | dLv] operand is produced in this
// launch by the deferred latent backward (LatRed): its loads wait for the counter and are sc1.
// gate (the deferred dW2 workers, latent.hpp enc_latent16_w2_kernel): a device flag read at
// entry, whose 0 drops the tile before its stores -- the operand loads go out speculatively
// instead of one scalar round trip after it.
template <bool VEC, int NWV, int TS, bool DA3 = false, bool DEFER = false, class WA>
DEV void wgrad_body(const WA& p, const WGroup& g, int bid, float (*sa)[kWP], float (*sb)[kWP],
                    const int* gate = nullptr) {
    const int gv = gate ? ld_launch_const(gate) : 1;
    static_assert(NWV == 4 || NWV == 8, "wgrad: 4 or 8 waves");
    static_assert(TS == 1 || TS == 2 || TS == 4, "wgrad: 16, 32 or 64 columns per tile");
    constexpr int kWTS = TS, kWTJ = 16 * TS;
    constexpr int NTH = 64 * NWV;
    // the thread's index in its tile worker (a 1024-thread workgroup can run two 512-thread
    // workers side by side: enc_latent16_w2_kernel)
    const int tid = (int)threadIdx.x % NTH;
    // resolve the batch pointer first: its load must not queue behind the prefetches below
    const float* at = g.at_is_x ? wa_xbase(p) + (int64_t)ld_launch_const(wa_cur_batch(p)) * wa_batch_stride(p) : g.at;
    const rsrc_t ba = mkbuf(at, (int64_t)g.klim_at * g.ld_at * 4);
#ifdef VAEB_TIMELINE
    if (VAEB_DBG_ON(p.dbg) && tid == 0) {   // the batch pointer resolved
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        p.dbg[bid * 8 + 4] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    const int lt = bid - g.wg_begin;
    const int i0 = (lt / g.tiles_j) * kWT, j0 = (lt % g.tiles_j) * kWTJ;
    const int lane = tid & 63, wave = (tid >> 6) & 3, kh = tid >> 8;
    const int li = lane & 15, q = lane >> 4;
    const int NT = g.N0 + g.N1;

    // ---- prefetch theta / acc of this lane's outputs.  TV (VEC -- the host also checked that
    // every group's arena offsets and widths are multiples of 4 -- and TS >= 2): the epilogue owns, per lane, four
    // consecutive columns j0 + 16 t + 4 (lane & 3) .. + 3 of row i0 + 16 w + (lane >> 2) -- the
    // accumulators are transposed through LDS -- so theta, the Adagrad state and the outputs
    // move as 16-byte accesses (one vector-memory instruction instead of four).  Else rows
    // i0 + 16 w + 4 q + r, column j0 + 16 t + li: the MFMA layout itself.
    const bool upd = p.opt.update != 0;
    const rsrc_t bth = mkbuf(p.opt.theta_in, p.P * 4), bac = mkbuf(p.opt.acc, p.P * 4);
    uint32_t off[kWTS][4];
    float th[kWTS][4], ac[kWTS][4];
    uint32_t off4[kWTS];
    f32x4 th4[kWTS], ac4[kWTS];
    // (measured on the 32-wide dW2 tiles of the dhd launch 11.95 -> 11.37 us; on the 16-wide
    // tiles of the last launch 9.77 -> 10.0 us, so those keep the MFMA layout)
    constexpr bool TV = VEC && !kNoTV && kWTS >= 2;
    if constexpr (TV) {
#pragma unroll
        for (int t = 0; t < kWTS; ++t) {
            const int j = j0 + 16 * t + 4 * (lane & 3);
            const bool s1 = j >= g.N0;
            const int jj = s1 ? j - g.N0 : j;
            const int nrow = s1 ? g.N1 : g.N0;
            const int i = i0 + 16 * wave + (lane >> 2);
            const bool ok = j < NT && i <= g.rowsW;
            const int64_t idx = (i < g.rowsW) ? (s1 ? g.offW1 : g.offW0) + (int64_t)i * nrow + jj
                                              : (s1 ? g.offb1 : g.offb0) + jj;
            off4[t] = ok ? (uint32_t)idx * 4u : kOOB;
            const uint32_t lo = (upd && kh == 0) ? off4[t] : kOOB;
            th4[t] = bld4(bth, lo);
            ac4[t] = bld4(bac, lo);
        }
    }
#pragma unroll
    for (int t = 0; t < (TV ? 0 : kWTS); ++t) {
        const int j = j0 + 16 * t + li;
        const bool s1 = j >= g.N0;
        const int jj = s1 ? j - g.N0 : j;
        const int nrow = s1 ? g.N1 : g.N0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + 16 * wave + 4 * q + r;
            const bool ok = j < NT && i <= g.rowsW;
            const int64_t idx = (i < g.rowsW) ? (s1 ? g.offW1 : g.offW0) + (int64_t)i * nrow + jj
                                              : (s1 ? g.offb1 : g.offb0) + jj;
            off[t][r] = ok ? (uint32_t)idx * 4u : kOOB;
            // unconditional loads (no branch): the waitcnt pass then sees them retired
            // by the first panel wait instead of re-waiting after every epilogue store
            uint32_t lo = (upd && kh == 0) ? off[t][r] : kOOB;
            th[t][r] = bld(bth, lo);
            ac[t][r] = bld(bac, lo);
        }
    }

    // ---- K loop over LDS stages of kWKB rows
    const rsrc_t bb0 = mkbuf(g.b0, (int64_t)g.K * g.ld0 * 4);
    const rsrc_t bb1 = mkbuf(g.b1 ? g.b1 : g.b0, (int64_t)g.K * (g.b1 ? g.ld1 : g.ld0) * 4);
    // VEC (chosen on the host): every panel row is 16-byte aligned with widths % 4 == 0
    constexpr bool va = VEC, vb = VEC;
    f32x4 acc[kWTS];
#pragma unroll
    for (int t = 0; t < kWTS; ++t) acc[t] = zero4();
    int kb = 0;
    do {  // K >= 1 always; a do-loop keeps the pre-loop loads off the exit path
        // stage the panels: element e = (row kr, float4 column c4).  All 16 loads of a
        // thread are issued before the first LDS store (one memory round trip).
        constexpr int NU = (kWKB * 16) / NTH;
        f32x4 ra[NU], rb[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int e = tid + NTH * u;
            const int kr = e >> 4, c4 = e & 15;
            const int k = kb + kr;
            const int i = i0 + 4 * c4, j = j0 + 4 * c4;
            const bool jt = 4 * c4 < kWTJ;   // B columns beyond a narrow tile: no fetch
            if (va) {
                ra[u] = bld4(ba, (k < g.klim_at && i < g.rowsW) ? (uint32_t)(k * g.ld_at + i) * 4u : kOOB);
            } else {
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    ra[u][s] = bld(ba, (k < g.klim_at && i + s < g.rowsW) ? (uint32_t)(k * g.ld_at + i + s) * 4u : kOOB);
            }
            if (DA3 || DEFER) {
                rb[u] = zero4();   // (DEFER: loaded below, after the counter poll)
            } else if (vb) {
                const bool in0 = j < g.N0;
                const uint32_t o0 = (jt && k < g.K && in0) ? (uint32_t)(k * g.ld0 + j) * 4u : kOOB;
                const uint32_t o1 = (jt && k < g.K && !in0 && j - g.N0 < g.N1) ? (uint32_t)(k * g.ld1 + j - g.N0) * 4u : kOOB;
                rb[u] = in0 ? bld4(bb0, o0) : bld4(bb1, o1);
            } else {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int jj = j + s;
                    const bool in0 = jj < g.N0;
                    rb[u][s] = in0 ? bld(bb0, (jt && k < g.K) ? (uint32_t)(k * g.ld0 + jj) * 4u : kOOB)
                                   : bld(bb1, (jt && k < g.K && jj - g.N0 < g.N1) ? (uint32_t)(k * g.ld1 + jj - g.N0) * 4u : kOOB);
                }
            }
        }
#ifdef VAEB_TIMELINE
        if (VAEB_DBG_ON(p.dbg) && kb == 0) {   // the stage's panel loads landed
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (tid == 0) p.dbg[bid * 8 + 5] = __builtin_amdgcn_s_memrealtime();
        }
#endif
        if constexpr (DEFER && !DA3) {
            // B panel = [dMu | dLv] of this launch's reducers: poll, then sc1 loads only
            // (the counter replica of this workgroup's round-robin slot)
            if (kb == 0) lat_wait(p.hd.red_cnt + lat_slot() * kLatCntStride, p.hd.nred, &p.da3.red.guard);
            const rsrc_t cb0 = bb0, cb1 = bb1;
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int e = tid + NTH * u;
                const int kr = e >> 4, c4 = e & 15;
                const int k = kb + kr;
                const int j = j0 + 4 * c4;
                const bool jt = 4 * c4 < kWTJ;
                if (vb) {
                    const bool in0 = j < g.N0;
                    const uint32_t o0 = (jt && k < g.K && in0) ? (uint32_t)(k * g.ld0 + j) * 4u : kOOB;
                    const uint32_t o1 = (jt && k < g.K && !in0 && j - g.N0 < g.N1) ? (uint32_t)(k * g.ld1 + j - g.N0) * 4u : kOOB;
                    rb[u] = in0 ? bld4x<16>(cb0, o0) : bld4x<16>(cb1, o1);
                } else {
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        const int jj = j + s;
                        const bool in0 = jj < g.N0;
                        rb[u][s] = in0 ? bldx<16>(cb0, (jt && k < g.K) ? (uint32_t)(k * g.ld0 + jj) * 4u : kOOB)
                                       : bldx<16>(cb1, (jt && k < g.K && jj - g.N0 < g.N1) ? (uint32_t)(k * g.ld1 + jj - g.N0) * 4u : kOOB);
                    }
                }
            }
        }
        if constexpr (DA3 && DEFER)
            da3_panel<NWV, TS, true>(p.da3, kb, j0, i0 == 0, sb, p.hd.red_cnt, p.hd.nred,
                                     VAEB_DBG_ON(p.dbg) ? p.dbg + bid * 8 : nullptr);
        else if constexpr (DA3) da3_panel<NWV, TS>(p.da3, kb, j0, i0 == 0, sb);
#ifdef VAEB_TIMELINE
        if (VAEB_DBG_ON(p.dbg) && kb == 0 && tid == 0) p.dbg[bid * 8 + 2] = __builtin_amdgcn_s_memrealtime();
#endif
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int e = tid + NTH * u;
            const int kr = e >> 4, c4 = e & 15;
            const int i = i0 + 4 * c4;
            // the all-ones row (bias gradient) for every batch row of the padded K
            f32x4 v = ra[u];
#pragma unroll
            for (int s = 0; s < 4; ++s) v[s] = (i + s == g.rowsW) ? ((kb + kr < g.K) ? 1.f : 0.f) : v[s];
            *reinterpret_cast<f32x4*>(&sa[kr][4 * c4]) = v;
            if constexpr (!DA3) *reinterpret_cast<f32x4*>(&sb[kr][4 * c4]) = rb[u];
        }
        __syncthreads();
#ifdef VAEB_TIMELINE
        if (VAEB_DBG_ON(p.dbg) && kb == 0 && tid == 0) p.dbg[bid * 8 + 6] = __builtin_amdgcn_s_memrealtime();
#endif
        const int nch = min(kWKB, g.K - kb) >> 4;
        for (int c = kh; c < nch; c += NWV / 4) {
            const int kk = 16 * c + 4 * q;
            f32x4 a4;
#pragma unroll
            for (int s = 0; s < 4; ++s) a4[s] = sa[kk + s][16 * wave + li];
#pragma unroll
            for (int t = 0; t < kWTS; ++t) {
                f32x4 b4;
#pragma unroll
                for (int s = 0; s < 4; ++s) b4[s] = sb[kk + s][16 * t + li];
                acc[t] = mfma4(a4, b4, acc[t]);
            }
        }
        __syncthreads();
        kb += kWKB;
    } while (kb < g.K);
    if constexpr (NWV == 8) {  // fold the odd-chunk half into waves 0..3 (sa is free again)
        f32x4* red = reinterpret_cast<f32x4*>(&sa[0][0]);
        if (kh == 1)
#pragma unroll
            for (int t = 0; t < kWTS; ++t) red[(wave * 4 + t) * 64 + lane] = acc[t];
        __syncthreads();
        if (kh == 1) return;
#pragma unroll
        for (int t = 0; t < kWTS; ++t) acc[t] += red[(wave * 4 + t) * 64 + lane];
    }
    if (VAEB_DBG_ON(p.dbg) && tid == 0) p.dbg[bid * 8 + 1] = __builtin_amdgcn_s_memrealtime();
    if (gv == 0) return;   // (wave-uniform; no barrier follows)

    // ---- epilogue: out-of-range byte offsets make masked buffer stores no-ops
    const rsrc_t bto = mkbuf(p.opt.theta_out, p.P * 4), bgr = mkbuf(p.opt.grad, p.P * 4);
    if constexpr (TV) {
        // transpose the wave's 16 x 16 TS accumulator block through its own LDS region (sb is
        // free: the last stage's barrier retired every panel read; a wave reads only what it
        // wrote, in order)
        constexpr int TP = 16 * kWTS + 1;
        float* tl = &sb[0][0] + wave * 16 * TP;
#pragma unroll
        for (int t = 0; t < kWTS; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) tl[(4 * q + r) * TP + 16 * t + li] = acc[t][r];
#pragma unroll
        for (int t = 0; t < kWTS; ++t) {
            f32x4 gv, nt4, a4 = ac4[t];
#pragma unroll
            for (int c = 0; c < 4; ++c) gv[c] = tl[(lane >> 2) * TP + 16 * t + 4 * (lane & 3) + c];
            if (p.opt.store_grad)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, gv), bgr, off4[t], 0, 0);
            if (upd) {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    float a2 = a4[c];
                    nt4[c] = opt_rule(p.opt, th4[t][c], a2, gv[c]);
                    a4[c] = a2;
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, a4), bac, off4[t], 0, kStWT);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, nt4), bto, off4[t], 0, kStWT);
            }
        }
        if (VAEB_DBG_ON(p.dbg) && tid == 0) p.dbg[bid * 8 + 3] = __builtin_amdgcn_s_memrealtime();
        return;
    }
#pragma unroll
    for (int t = 0; t < kWTS; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float dsg = acc[t][r];
            if (p.opt.store_grad) bst(bgr, off[t][r], dsg);
            if (upd) {
                float a2 = ac[t][r];
                const float nt = opt_rule(p.opt, th[t][r], a2, dsg);
                bst_opt(bac, off[t][r], a2);
                bst_opt(bto, off[t][r], nt);
            }
        }
    if (VAEB_DBG_ON(p.dbg) && tid == 0) p.dbg[bid * 8 + 3] = __builtin_amdgcn_s_memrealtime();
}

template <bool VEC, int TS>
__global__ __launch_bounds__(256) void wgrad_kernel(WGradArgs p) {
    __shared__ float sa[kWKB][kWP];
    __shared__ float sb[kWKB][kWP];
    // the ELBO workgroup (with_elbo) is block 0, dispatched first, so its reduction runs
    // beside the weight-gradient tiles instead of after the last of them was placed
    int bid;
    if (p.with_elbo)
        bid = blockIdx.x == 0 ? p.total_wgs : xcd_remap((int)blockIdx.x - 1, p.total_wgs);
    else
        bid = (int)blockIdx.x < p.total_wgs ? xcd_remap(blockIdx.x, p.total_wgs) : (int)blockIdx.x;
    if (VAEB_DBG_ON(p.dbg) && threadIdx.x == 0) p.dbg[bid * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    if (bid >= p.total_wgs) {  // the extra workgroup: ELBO of this step
        elbo_reduce(p.elbo, reinterpret_cast<double*>(&sa[0][0]));
        return;
    }
    if (p.ngroups > 1 && bid >= p.g[1].wg_begin) wgrad_body<VEC, 4, TS>(p, p.g[1], bid, sa, sb);
    else wgrad_body<VEC, 4, TS>(p, p.g[0], bid, sa, sb);
}

// The deferred dW2's flush (vaeb_hip.hip w2_flush): the pending step's dW2 (| dW6) tiles as
// their own launch, when the host reads or replaces the state before another step ran them.
// (512-thread tiles, as in the encoder launch: the same K split, so the same sums bit for bit)
template <bool VEC, int TS>
__global__ __launch_bounds__(512) void w2_flush_kernel(WGradArgs p, const int* pend) {
    __shared__ float sa[kWKB][kWP];
    __shared__ float sb[kWKB][kWP];
    if (ld_launch_const(pend) == 0) return;
    wgrad_body<VEC, 8, TS>(p, p.g[0], xcd_remap(blockIdx.x, p.total_wgs), sa, sb);
}

// The folded latent backward's last launch: dW3 (dA3 formed in the workgroup) | dW4 | dW5
// | dW1, and the ELBO workgroup first.  VM: bit g = group g's panels take 16-byte loads.
// DEFER (LatRed, p.da3.red.nred reducers): blocks [ELBO][reducers][tiles], the reducers
// dispatched ahead of every tile that waits for them (and 2 workgroups per CU hold the whole
// grid at MNIST: 1 + 21 + 448 <= 512).  Stamps: reducers at logical ids total_wgs + 1 + r.
template <int VM, int TS, bool DEFER>
__global__ __launch_bounds__(256) void wgrad3_kernel(WGradArgs3 p) {
    __shared__ float sa[kWKB][kWP];
    __shared__ float sb[kWKB][kWP];
    const W3Head h = p.hd;   // one scalar load: the role and group boundaries
    // (the empty asm makes every field live here, so the loads go out together, before the
    // first branch, instead of one dependent round trip per branch)
    asm volatile("" ::"s"(h.with_elbo), "s"(h.total_wgs), "s"(h.nred), "s"(h.gb1), "s"(h.gb2), "s"(h.xbase),
                 "s"(h.cur_batch), "s"(h.batch_stride), "s"(h.red_cnt));
    int b = (int)blockIdx.x;
    if (h.with_elbo) {
        if (b == 0) {
            if (VAEB_DBG_ON(p.dbg) && threadIdx.x == 0) p.dbg[h.total_wgs * 8 + 0] = __builtin_amdgcn_s_memrealtime();
            elbo_reduce(p.elbo, reinterpret_cast<double*>(&sa[0][0]));
            return;
        }
        --b;
    }
    if constexpr (DEFER) {
        if (b < h.nred) {
            const int sid = h.total_wgs + 1 + b;
            if (VAEB_DBG_ON(p.dbg) && threadIdx.x == 0) p.dbg[sid * 8 + 0] = __builtin_amdgcn_s_memrealtime();
            lat_reduce_wg(p.da3.red, b, reinterpret_cast<f32x4*>(&sa[0][0]), reinterpret_cast<float(*)[17]>(&sb[0][0]),
                          VAEB_DBG_ON(p.dbg) ? p.dbg + sid * 8 : nullptr);
            if (VAEB_DBG_ON(p.dbg) && threadIdx.x == 0) p.dbg[sid * 8 + 3] = __builtin_amdgcn_s_memrealtime();
            return;
        }
        b -= h.nred;
    }
    const int bid = xcd_remap(b, h.total_wgs);
    if (VAEB_DBG_ON(p.dbg) && threadIdx.x == 0) p.dbg[bid * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    if (bid >= h.gb2) {
        wgrad_body<(VM & 4) != 0, 4, TS>(p, p.g[2], bid, sa, sb);
    } else if (bid >= h.gb1) {
        wgrad_body<(VM & 2) != 0, 4, TS, false, DEFER>(p, p.g[1], bid, sa, sb);
    } else {
        wgrad_body<(VM & 1) != 0, 4, TS, true, DEFER>(p, p.g[0], bid, sa, sb);
    }
}

// ----------------------------------------------------------------- DP optimizer
// After the RCCL all-reduce of [grad arena | SGVB]: replicated Adagrad with the prior
// added once (so every rank applies the identical update).  The arena is reduced in two
// buckets (vaeb_hip.hip: dp_bucket_*): a DpRange names the arena elements one launch
// updates, as up to two index runs [lo0, lo0 + n0) and [lo1, lo1 + n1); `book` = this
// launch also publishes the step's SGVB and advances the cursor / step counter.
// Up to kDpRuns index runs [lo[k], lo[k] + n[k]) -- sharded DP (vaeb_hip.hip dp_reduce_update):
// this rank's shard and the replicated tail of each of the arena's three runs.
constexpr int kDpRuns = 6;
struct DpRange {
    int64_t lo[kDpRuns], n[kDpRuns];
    int book;
    DEV int64_t total() const {
        int64_t t = 0;
#pragma unroll
        for (int k = 0; k < kDpRuns; ++k) t += n[k];
        return t;
    }
    DEV int64_t at(int64_t v) const {
#pragma unroll
        for (int k = 0; k < kDpRuns - 1; ++k) {
            if (v < n[k]) return lo[k] + v;
            v -= n[k];
        }
        return lo[kDpRuns - 1] + v;
    }
};
__global__ __launch_bounds__(256) void adagrad_kernel(OptArgs o, int64_t P, DpRange r, ElboArgs e) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t n = r.total();
    const rsrc_t bti = mkbuf(o.theta_in, P * 4), bto = mkbuf(o.theta_out, P * 4);
    const rsrc_t bac = mkbuf(o.acc, P * 4), bgr = mkbuf(o.grad, P * 4);
    // U grid-stride elements per memory round trip: every load is issued before any store
    // (hipcc cannot reorder a per-element load -> store chain: the arrays may alias)
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
            float a = ac[u];
            const float tn = opt_rule(o, th[u], a, gr[u]);
            bst_opt(bto, off[u], tn);
            bst_opt(bac, off[u], a);
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

// ------------------------------------------------ full variational, weight sampling
// VAEB_EST_FVS (extension): the weight-posterior reparameterisation of
// VAEB.sample_variational_params (VAEB.py:127-129), theta~ = mu + |sigma| zeta, used by the
// data term of getFVBL (VAEB.py:349-367); criterion as the literal path (VAEB.py:386-399).
// zeta: host buffer, or Philox keyed by (seed, step, parameter index) on a counter range
// disjoint from the latent noise (c1 bit 30).
// One Philox block per 16-byte group g of parameters: both Box-Muller pairs of its four
// outputs give the group's four normals.
DEV f32x4 fvs_zeta4(int64_t g, uint64_t seed, int64_t step) {
    uint32_t ctr[4] = {(uint32_t)g, 0x40000000u | (uint32_t)(g >> 32), 0u, 0u};
    const uint64_t c23 = philox_c23(step, 0);
    ctr[2] = (uint32_t)c23;
    ctr[3] = (uint32_t)(c23 >> 32);
    philox4x32(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float r0 = __builtin_amdgcn_sqrtf(-2.0f * flog(((float)(ctr[0] >> 8) + 1.0f) * (1.0f / 16777216.0f)));
    const float r1 = __builtin_amdgcn_sqrtf(-2.0f * flog(((float)(ctr[2] >> 8) + 1.0f) * (1.0f / 16777216.0f)));
    const float t0 = (float)(ctr[1] >> 8) * (1.0f / 16777216.0f);   // revolutions
    const float t1 = (float)(ctr[3] >> 8) * (1.0f / 16777216.0f);
    f32x4 z;
    z[0] = r0 * __builtin_amdgcn_cosf(t0);
    z[1] = r0 * __builtin_amdgcn_sinf(t0);
    z[2] = r1 * __builtin_amdgcn_cosf(t1);
    z[3] = r1 * __builtin_amdgcn_sinf(t1);
    return z;
}
DEV float fvs_zeta(int64_t i, const float* zin, uint64_t seed, int64_t step) {
    if (zin) return zin[i];
    return fvs_zeta4(i >> 2, seed, step)[i & 3];
}
// The (mu, sigma) streams below move 16-byte groups: thread t of the grid takes groups
// t, t + T, ... (U per round trip, every load before any store), the P % 4 tail elements
// go to threads 0..2 of block 0.  kFvGrid x 256 threads x U x 4 elements cover MNIST's
// 0.8 M parameters in one round trip.
DEV void fv_group(int64_t g, int64_t n4, uint32_t& off) { off = g < n4 ? (uint32_t)(g * 16) : kOOB; }
// 16-byte stores of the FV / FVS parameter streams: written through like bst_opt (FV step
// 28.6 -> 28.2 us, fvs_update 9.4 -> 8.0 us)
DEV void bst4(rsrc_t b, uint32_t off, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), b, off, 0, kStWT);
}

__global__ __launch_bounds__(256) void fvs_sample_kernel(const float* mu, const float* sg, float* theta, int64_t P,
                                                        uint64_t seed, const int64_t* step, const float* zin) {
    const int64_t T = (int64_t)gridDim.x * 256, n4 = P >> 2;
    const int64_t stp = *step;
    const rsrc_t bm = mkbuf(mu, P * 4), bs = mkbuf(sg, P * 4), bt = mkbuf(theta, P * 4);
    const rsrc_t bz = mkbuf(zin, zin ? P * 4 : 0);
    constexpr int U = 2;
    for (int64_t g0 = (int64_t)blockIdx.x * 256 + threadIdx.x; g0 < n4; g0 += U * T) {
        uint32_t off[U];
        f32x4 m[U], s[U], z[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            fv_group(g0 + u * T, n4, off[u]);
            m[u] = bld4(bm, off[u]);
            s[u] = bld4(bs, off[u]);
            z[u] = bld4(bz, zin ? off[u] : kOOB);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (off[u] == kOOB) continue;
            const f32x4 zz = zin ? z[u] : fvs_zeta4(g0 + u * T, seed, stp);
            f32x4 t;
#pragma unroll
            for (int k = 0; k < 4; ++k) t[k] = m[u][k] + fabsf(s[u][k]) * zz[k];
            bst4(bt, off[u], t);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (P & 3)) {
        const int64_t i = n4 * 4 + threadIdx.x;
        theta[i] = mu[i] + fabsf(sg[i]) * fvs_zeta(i, zin, seed, stp);
    }
}

// Given the data gradient G = d(sum log p + sum KL)/d theta~ at the sample (grad arena):
//   d/dmu    = B G - 2 mu                                  (thetaPrior -mu, L2 -mu)
//   d/dsigma = B G zeta sign(sigma) + 1/sigma - 2 sigma    (thetaPrior 1/sigma - sigma, L2 -sigma)
// then Adagrad on both (VAEB.py:426-444); thetaPrior partials from the pre-update values.
// next_theta (Philox mode): also writes the next step's sample mu' + |sigma'| zeta(step + 1),
// so a graph-replayed sequence draws it once, at its first step.
struct FvsElem {
    float B, lr, eps;
    DEV void operator()(float& m, float& s, float& a1, float& a2, float G, float zz, double& tp) const {
        tp += 0.5 * (1.0 + (double)logf(s * s) - (double)m * m - (double)s * s);
        const float gm = B * G - 2.f * m;
        const float gs = B * G * zz * (s >= 0.f ? 1.f : -1.f) + 1.f / s - 2.f * s;
        a1 += gm * gm;
        a2 += gs * gs;
        m += lr * gm / (sqrtf(a1) + eps);
        s += lr * gs / (sqrtf(a2) + eps);
    }
};
__global__ __launch_bounds__(256) void fvs_update_kernel(float* mu, float* sg, float* am, float* as, const float* grad,
                                                        int64_t P, float B, float lr, float eps, uint64_t seed,
                                                        const int64_t* step, const float* zin, float* part,
                                                        float* next_theta) {
    __shared__ double sh[256];
    double tp = 0;
    const FvsElem f{B, lr, eps};
    const rsrc_t bn = mkbuf(next_theta, next_theta ? P * 4 : 0);
    const int64_t T = (int64_t)gridDim.x * 256, n4 = P >> 2;
    const int64_t stp = *step;
    const rsrc_t bm = mkbuf(mu, P * 4), bs = mkbuf(sg, P * 4), bam = mkbuf(am, P * 4), bas = mkbuf(as, P * 4);
    const rsrc_t bg = mkbuf(grad, P * 4), bz = mkbuf(zin, zin ? P * 4 : 0);
    constexpr int U = 2;
    for (int64_t g0 = (int64_t)blockIdx.x * 256 + threadIdx.x; g0 < n4; g0 += U * T) {
        uint32_t off[U];
        f32x4 m[U], s[U], a1[U], a2[U], G[U], z[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            fv_group(g0 + u * T, n4, off[u]);
            m[u] = bld4(bm, off[u]);
            s[u] = bld4(bs, off[u]);
            a1[u] = bld4(bam, off[u]);
            a2[u] = bld4(bas, off[u]);
            G[u] = bld4(bg, off[u]);
            z[u] = bld4(bz, zin ? off[u] : kOOB);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (off[u] == kOOB) continue;
            const f32x4 zz = zin ? z[u] : fvs_zeta4(g0 + u * T, seed, stp);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float mm = m[u][k], ss = s[u][k], x1 = a1[u][k], x2 = a2[u][k];
                f(mm, ss, x1, x2, G[u][k], zz[k], tp);
                m[u][k] = mm; s[u][k] = ss; a1[u][k] = x1; a2[u][k] = x2;
            }
            bst4(bam, off[u], a1[u]);
            bst4(bas, off[u], a2[u]);
            bst4(bm, off[u], m[u]);
            bst4(bs, off[u], s[u]);
            if (next_theta) {   // the next step's sample (Philox mode; fvs_sample_kernel's rule)
                const f32x4 zn = fvs_zeta4(g0 + u * T, seed, stp + 1);
                f32x4 t;
#pragma unroll
                for (int k = 0; k < 4; ++k) t[k] = m[u][k] + fabsf(s[u][k]) * zn[k];
                bst4(bn, off[u], t);
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (P & 3)) {
        const int64_t i = n4 * 4 + threadIdx.x;
        f(mu[i], sg[i], am[i], as[i], grad[i], fvs_zeta(i, zin, seed, stp), tp);
        if (next_theta) next_theta[i] = mu[i] + fabsf(sg[i]) * fvs_zeta(i, nullptr, seed, stp + 1);
    }
    tp = block_sum256w(tp, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = (float)tp;
}

// ----------------------------------------------------------------- full variational
// Literal --full_varational update (VAEB.py:117-125, 349-367, 392-393, 426-444):
// g_mu = -2 mu, g_sigma = 1/sigma - 2 sigma; thetaPrior partials from pre-update values.
struct FvElem {
    float lr, eps;
    int update;
    DEV void operator()(float& m, float& s, float& a1, float& a2, double& tp) const {
        tp += 0.5 * (1.0 + (double)logf(s * s) - (double)m * m - (double)s * s);
        if (!update) return;
        const float gm = -2.f * m;
        const float gs = 1.f / s - 2.f * s;
        a1 += gm * gm;
        a2 += gs * gs;
        m += lr * gm / (sqrtf(a1) + eps);
        s += lr * gs / (sqrtf(a2) + eps);
    }
};
__global__ __launch_bounds__(256) void fv_kernel(float* mu, float* sg, float* am, float* as, int64_t P,
                                                 float lr, float eps, int update, float* part) {
    __shared__ double sh[256];
    double tp = 0;
    const FvElem f{lr, eps, update};
    const int64_t T = (int64_t)gridDim.x * 256, n4 = P >> 2;
    const rsrc_t bm = mkbuf(mu, P * 4), bs = mkbuf(sg, P * 4), bam = mkbuf(am, P * 4), bas = mkbuf(as, P * 4);
    constexpr int U = 2;   // 16-byte groups per round trip (fvs_sample_kernel's scheme)
    for (int64_t g0 = (int64_t)blockIdx.x * 256 + threadIdx.x; g0 < n4; g0 += U * T) {
        uint32_t off[U];
        f32x4 m[U], s[U], a1[U], a2[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            fv_group(g0 + u * T, n4, off[u]);
            m[u] = bld4(bm, off[u]);
            s[u] = bld4(bs, off[u]);
            a1[u] = bld4(bam, update ? off[u] : kOOB);
            a2[u] = bld4(bas, update ? off[u] : kOOB);
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
            if (update) {
                bst4(bam, off[u], a1[u]);
                bst4(bas, off[u], a2[u]);
                bst4(bm, off[u], m[u]);
                bst4(bs, off[u], s[u]);
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (P & 3)) {
        const int64_t i = n4 * 4 + threadIdx.x;
        float m = mu[i], s = sg[i], a1 = update ? am[i] : 0.f, a2 = update ? as[i] : 0.f;
        f(m, s, a1, a2, tp);
        if (update) { mu[i] = m; sg[i] = s; am[i] = a1; as[i] = a2; }
    }
    tp = block_sum256w(tp, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = (float)tp;
}

}  // namespace vaeb
