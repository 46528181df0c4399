// fused.hpp -- the two latent-width phases of the SGVB step as single launches, one
// 512-thread workgroup per 16 batch rows (requires Z <= 32; larger Z uses the generic
// tile phases of phases.hpp).
//
//  heads_dechid_kernel (P23):
//     [mu | lv] = h [W4 | W5] + [b4 | b5]            VAEB.py:248-249  (K = H, 8-way K split)
//     eps, z = mu + exp(lv/2) eps, KL or prior-logQ   VAEB.py:41-47, 343 / 322-325
//     hd = tanh(z W1 + b1)                            VAEB.py:254      (z kept in LDS)
//  dz_dh_kernel (P67):
//     dZ = dA1 W1^T                                   (K = H, 8-way K split)
//     [dMu | dLv] from dZ (summed over the L samples), mu, lv, eps, z  
//     dA3 = ([dMu | dLv] [W4 | W5]^T) * (1 - h^2)     ([dMu|dLv] kept in LDS)
//
// A dependent global round trip costs ~1 us here (measured with VAEB_STAMP), so both
// kernels issue EVERY global operand they will need -- GEMM operands of both stages,
// biases, eps, mu/lv, h -- at entry, before the first MFMA; the element-wise middle
// stage is spread over all 512 threads (one (row, latent) element each).
#pragma once
#include "phases.hpp"

namespace vaeb {

constexpr int kZP = 32;   // LDS row pitch of z tiles (Z <= 32); thread t owns (t >> 5, t & 31)
constexpr int kKP = 64;   // LDS row pitch of [dMu | dLv] (2Z <= 64)
constexpr int kLP = 4;    // samples whose per-element operands are prefetched / kept in LDS

// Sum over the 32 lanes that share t >> 5 (one latent row).
DEV float sum32(float v) {
    v = sum16(v);
    v += __shfl_xor(v, 16, 64);
    return v;
}

// ---------------------------------------------------------------------------- P23
template <int NCT>
__global__ __launch_bounds__(512) void heads_dechid_kernel(StepArgs a) {
    __shared__ f32x4 red[8][2 * NCT][64];
    __shared__ float zs[kLP][16][kZP];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, q = lane >> 4;
    const int i0 = blockIdx.x * 16;
    const int Z = a.Z, H = a.H;
    VAEB_STAMP(a, 0);

    // ---- prefetch: element-wise operands of this thread's (row, latent) element
    const int ml = threadIdx.x >> 5, n = threadIdx.x & 31;
    const int m = i0 + ml;
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
    const int64_t grow0 = global_row0(a);
    const int64_t stp = a.step ? *a.step : 0;
    // ---- prefetch: stage-2 operands (W1 columns, b1) of this wave's first 4 tiles
    const rsrc_t bw1 = mkbuf(a.W1, (int64_t)Z * H * 4);
    const rsrc_t bb1 = mkbuf(a.b1, (int64_t)H * 4);
    const int nctH = (H + 15) >> 4;
    const int ntiles = a.L * nctH;
    f32x4 w1pre[4][NCT];
    float b1pre[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int nn = ((wave + 8 * u) % nctH) * 16 + li;
#pragma unroll
        for (int c = 0; c < NCT; ++c) w1pre[u][c] = mc4(bw1, H, nn, c * 16 + 4 * q, H, Z);
        b1pre[u] = bld(bb1, nn < H ? (uint32_t)nn * 4u : kOOB);
    }

    // ---- stage 1: [mu|lv] for 16 rows, K = H split over 8 waves
    f32x4 acc[2 * NCT];
#pragma unroll
    for (int w = 0; w < 2 * NCT; ++w) acc[w] = zero4();
    {
        const rsrc_t bh = mkbuf(a.h, (int64_t)a.Mbp * H * 4);
        const rsrc_t bw4 = mkbuf(a.W4, (int64_t)H * Z * 4);
        const rsrc_t bw5 = mkbuf(a.W5, (int64_t)H * Z * 4);
        const bool vh = (H & 3) == 0;
        const int nch = (H + 15) >> 4;
        for (int c0 = wave; c0 < nch; c0 += 8 * 4) {
            f32x4 av[4], bv[4][2 * NCT];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = (c0 + 8 * u) * 16 + 4 * q;
                av[u] = kc4(bh, H, i0 + li, k, a.Mbp, H, vh);
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) {
                    bv[u][2 * ct] = mc4(bw4, Z, ct * 16 + li, k, Z, H);
                    bv[u][2 * ct + 1] = mc4(bw5, Z, ct * 16 + li, k, Z, H);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int w = 0; w < 2 * NCT; ++w) acc[w] = mfma4(av[u], bv[u][w], acc[w]);
        }
    }
    VAEB_STAMP(a, 1);
#pragma unroll
    for (int w = 0; w < 2 * NCT; ++w) red[wave][w][lane] = acc[w];
    __syncthreads();
    VAEB_STAMP(a, 2);

    // ---- element-wise middle: thread (ml, n) -- mu, lv, eps, z, KL / LA terms
    {
        const int ct = n >> 4;
        const int src = (ml >> 2) * 16 + (n & 15), r = ml & 3;
        float mu = 0.f, lv = 0.f;
        if (ct < NCT) {
#pragma unroll
            for (int s = 0; s < 8; ++s) { mu += red[s][2 * ct][src][r]; lv += red[s][2 * ct + 1][src][r]; }
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
            if (l < kLP) zs[l][ml][n] = z;
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
    }
    VAEB_STAMP(a, 3);
    __syncthreads();
    VAEB_STAMP(a, 4);

    // ---- stage 2: hd = tanh(z W1 + b1) for (l, 16 rows) x H columns, K = Z (<= 2 chunks)
    auto tile2 = [&](int t, const f32x4 (&bw)[NCT], float b) {
        const int l = t / nctH, ct = t % nctH;
        const int nn = ct * 16 + li;
        f32x4 acc2 = zero4();
#pragma unroll
        for (int c = 0; c < NCT; ++c) {
            const int k = c * 16 + 4 * q;
            f32x4 av;
            if (l < kLP) av = *reinterpret_cast<const f32x4*>(&zs[l][li][k]);
            else av = kc4(mkbuf(a.z, (int64_t)a.Me * Z * 4), Z, l * a.Mbp + i0 + li, k, a.Me, Z, false);
            acc2 = mfma4(av, bw[c], acc2);
        }
        if (nn < H) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mm = i0 + 4 * q + r;
                a.hd[((int64_t)l * a.Mbp + mm) * H + nn] = (mm < a.Mb) ? ftanh(acc2[r] + b) : 0.f;
            }
        }
    };
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int t = wave + 8 * u;
        if (t < ntiles && t < nctH) tile2(t, w1pre[u], b1pre[u]);
    }
    for (int t = wave; t < ntiles; t += 8) {
        if (t < nctH && t < wave + 32) continue;  // done above with prefetched operands
        f32x4 bw[NCT];
        const int nn = (t % nctH) * 16 + li;
#pragma unroll
        for (int c = 0; c < NCT; ++c) bw[c] = mc4(bw1, H, nn, c * 16 + 4 * q, H, Z);
        tile2(t, bw, bld(bb1, nn < H ? (uint32_t)nn * 4u : kOOB));
    }
    VAEB_STAMP(a, 5);
}

// ---------------------------------------------------------------------------- P67
// Column split: nsp workgroups share row block i0; each recomputes stages 1-2 (dZ and
// [dMu | dLv] need the whole K = H reduction, ~100 KB of operands) and runs stage 3 for
// its 1/nsp of the H columns only, so the per-CU operand stream on this critical-path
// phase falls from ~250 KB (stage-3 [W4|W5] and h for all H columns) to ~130 KB at nsp = 4.
// Split 0 alone stores dZ and [dMu | dLv].
template <int NCT>
DEV void dz_dh_body(const StepArgs& a, int i0, int sp, int nsp) {
    __shared__ f32x4 red[8][NCT][64];
    __shared__ float dml[16][kKP];     // [dMu | dLv] tile (A operand of the dA3 GEMM)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, q = lane >> 4;
    const int Z = a.Z, H = a.H;
    for (int e = threadIdx.x; e < 16 * kKP; e += 512) dml[e / kKP][e % kKP] = 0.f;

    // ---- prefetch: element-wise operands of this thread's (row, latent) element
    const int ml = threadIdx.x >> 5, j = threadIdx.x & 31;
    const int m = i0 + ml;
    const bool valid = j < Z && m < a.Mb;
    const uint32_t oj = valid ? (uint32_t)(m * Z + j) * 4u : kOOB;
    const float mu = bld(mkbuf(a.mu, (int64_t)a.Mbp * Z * 4), oj);
    const float lv = bld(mkbuf(a.lv, (int64_t)a.Mbp * Z * 4), oj);
    float epre[kLP], zpre[kLP];
    {
        const rsrc_t be = mkbuf(a.eps, (int64_t)a.Me * Z * 4);
        const rsrc_t bz = mkbuf(a.z, (int64_t)a.Me * Z * 4);
#pragma unroll
        for (int l = 0; l < kLP; ++l) {
            const uint32_t o = (valid && l < a.L) ? (uint32_t)((l * a.Mbp + m) * Z + j) * 4u : kOOB;
            epre[l] = bld(be, o);
            zpre[l] = (a.est == EST_LA) ? bld(bz, o) : 0.f;
        }
    }
    // ---- prefetch: stage-3 operands ([W4|W5]^T columns, h) of this wave's first 4 tiles
    const rsrc_t bw4 = mkbuf(a.W4, (int64_t)H * Z * 4);
    const rsrc_t bw5 = mkbuf(a.W5, (int64_t)H * Z * 4);
    const rsrc_t bhh = mkbuf(a.h, (int64_t)a.Mbp * H * 4);
    const int nctH = (H + 15) >> 4;
    const int tper = (nctH + nsp - 1) / nsp, t_lo = sp * tper, t_hi = min(nctH, t_lo + tper);
    const bool vz = (Z & 3) == 0 && aligned16(a.W4) && aligned16(a.W5);
    auto ldw45 = [&](int nn, int k) {
        if (vz) return (k < Z) ? kc4(bw4, Z, nn, k, H, Z, true) : kc4(bw5, Z, nn, k - Z, H, Z, true);
        f32x4 v;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kk = k + s;
            const bool ok = nn < H;
            v[s] = bld(bw4, (ok && kk < Z) ? (uint32_t)(nn * Z + kk) * 4u : kOOB) +
                   bld(bw5, (ok && kk >= Z && kk < 2 * Z) ? (uint32_t)(nn * Z + kk - Z) * 4u : kOOB);
        }
        return v;
    };
    auto ldh = [&](int nn) {
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int mm = i0 + 4 * q + r;
            v[r] = bld(bhh, (nn < H && mm < a.Mb) ? (uint32_t)(mm * H + nn) * 4u : kOOB);
        }
        return v;
    };
    f32x4 w45pre[4][2 * NCT], hpre[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int t = t_lo + wave + 8 * u;
        const int nn = t < t_hi ? t * 16 + li : H;   // H: out of range, no fetch
#pragma unroll
        for (int c = 0; c < 2 * NCT; ++c) w45pre[u][c] = ldw45(nn, c * 16 + 4 * q);
        hpre[u] = ldh(nn);
    }

    // ---- stage 1: dZ_l = dA1_l W1^T for each sample l (K = H split over 8 waves);
    //      thread (ml, j) accumulates sum_l dZ_l and sum_l dZ_l * eps_l in registers
    const bool vh = (H & 3) == 0 && aligned16(a.W1);
    const rsrc_t bd1 = mkbuf(a.dA1, (int64_t)a.Me * H * 4);
    const rsrc_t bw1 = mkbuf(a.W1, (int64_t)Z * H * 4);
    float dzsum = 0.f, dzes = 0.f;
    for (int l = 0; l < a.L; ++l) {
        f32x4 acc[NCT];
#pragma unroll
        for (int w = 0; w < NCT; ++w) acc[w] = zero4();
        const int nch = (H + 15) >> 4;
        const int row = l * a.Mbp + i0 + li;
        for (int c0 = wave; c0 < nch; c0 += 8 * 4) {
            f32x4 av[4], bv[4][NCT];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = (c0 + 8 * u) * 16 + 4 * q;
                av[u] = kc4(bd1, H, row, k, a.Me, H, (H & 3) == 0);
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) bv[u][ct] = kc4(bw1, H, ct * 16 + li, k, Z, H, vh);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int w = 0; w < NCT; ++w) acc[w] = mfma4(av[u], bv[u][w], acc[w]);
        }
#pragma unroll
        for (int w = 0; w < NCT; ++w) red[wave][w][lane] = acc[w];
        __syncthreads();
        {
            const int ct = j >> 4;
            const int src = (ml >> 2) * 16 + (j & 15), r = ml & 3;
            float dz = 0.f;
            if (ct < NCT) {
#pragma unroll
                for (int s = 0; s < 8; ++s) dz += red[s][ct][src][r];
            }
            dz = valid ? dz : 0.f;
            const float e = (l < kLP) ? epre[l] : (valid ? a.eps[((int64_t)l * a.Mbp + m) * Z + j] : 0.f);
            dzsum += dz;
            dzes += dz * e;
            if (j < Z && sp == 0) a.dZ[((int64_t)l * a.Mbp + m) * Z + j] = dz;
        }
        __syncthreads();
    }
    VAEB_STAMP(a, 1);

    // ---- stage 2: [dMu | dLv] (LA: direct terms of VAEB.py:322-325)
    if (j < Z) {
        const float sl = a.sc / (float)a.L;
        const float sd = fexp(0.5f * lv);
        float dmu = 0.f, dlv = 0.f;
        if (valid) {
            if (a.est == EST_LA) {
                float tm = 0.f, tv = 0.f;
                for (int l = 0; l < a.L; ++l) {
                    const int64_t ol = ((int64_t)l * a.Mbp + m) * Z + j;
                    const float z = (l < kLP) ? zpre[l] : a.z[ol];
                    const float e = (l < kLP) ? epre[l] : a.eps[ol];
                    tm += -z;
                    tv += 0.5f - 0.5f * z * sd * e;
                }
                dmu = dzsum + sl * tm;
                dlv = dzes * 0.5f * sd + sl * tv;
            } else {
                dmu = dzsum - a.sc * mu;
                dlv = dzes * 0.5f * sd + a.sc * 0.5f * (1.f - fexp(lv));
            }
        }
        dml[ml][j] = dmu;
        dml[ml][Z + j] = dlv;
        if (sp == 0) {
            a.dMuLv[(int64_t)m * 2 * Z + j] = dmu;
            a.dMuLv[(int64_t)m * 2 * Z + Z + j] = dlv;
        }
    }
    VAEB_STAMP(a, 2);
    __syncthreads();
    VAEB_STAMP(a, 3);

    // ---- stage 3: dA3 = ([dMu|dLv] [W4|W5]^T) * (1 - h^2), K = 2Z (<= 4 chunks)
    auto tile3 = [&](int t, const f32x4 (&bw)[2 * NCT], const f32x4& hv) {
        const int nn = t * 16 + li;
        f32x4 acc2 = zero4();
#pragma unroll
        for (int c = 0; c < 2 * NCT; ++c) {
            const f32x4 av = *reinterpret_cast<const f32x4*>(&dml[li][c * 16 + 4 * q]);
            acc2 = mfma4(av, bw[c], acc2);
        }
        if (nn < H) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mm = i0 + 4 * q + r;
                a.dA3[(int64_t)mm * H + nn] = (mm < a.Mb) ? acc2[r] * (1.f - hv[r] * hv[r]) : 0.f;
            }
        }
    };
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int t = t_lo + wave + 8 * u;
        if (t < t_hi) tile3(t, w45pre[u], hpre[u]);
    }
    for (int t = t_lo + wave + 32; t < t_hi; t += 8) {
        f32x4 bw[2 * NCT];
#pragma unroll
        for (int c = 0; c < 2 * NCT; ++c) bw[c] = ldw45(t * 16 + li, c * 16 + 4 * q);
        tile3(t, bw, ldh(t * 16 + li));
    }
    VAEB_STAMP(a, 4);
}

template <int NCT>
__global__ __launch_bounds__(512) void dz_dh_kernel(StepArgs a) {
    VAEB_STAMP(a, 0);
    dz_dh_body<NCT>(a, blockIdx.x * 16, 0, 1);
}

}  // namespace vaeb
