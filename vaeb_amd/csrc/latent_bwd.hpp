// latent_bwd.hpp -- the latent-width backward folded into the dhd launch (training step,
// Z <= 32): the backward counterpart of latent.hpp's encoder fold.
//
//  dhd_dz_body (one 16 x 16 tile of dA1, 8 waves splitting K = D (| 2D Gaussian)):
//      dA1 = (dA2 W2^T (+ dA6 W6^T)) (1 - hd^2)                         
//      and the tile's share of dZ = dA1 W1^T: its 16 x 16 dA1 block times the matching
//      16 columns of W1^T, published as a write-through partial slab; the LAST tile of each
//      16-row latent block (over the H column tiles and the L sample planes) sums the
//      slabs in fixed order (bitwise reproducible) and runs the element-wise latent
//      backward: dZ, [dMu | dLv] = (sum_l dZ_l - sc mu, 1/2 s sum_l dZ_l eps_l +
//      sc/2 (1 - e^lv)), or the LA direct terms (VAEB.py:315-346).
//
// dA3 = ([dMu | dLv] [W4 | W5]^T) (1 - h^2) is then formed inside the dW3 workgroups of the
// last launch (kernels_aux.hpp: da3_panel), so the former dz / dh launch -- 56 workgroups
// that each recomputed dZ from 72 KB of dA1 and W1 -- and its kernel boundary are gone.
//
// Slab hand-off: the encoder's form (latent.hpp arrive_last and the guide rule cited
// there): sc1 slab stores by wave 0 only, its vmcnt drain, one relaxed agent-scope ticket
// per tile on the row block's counter, sc1 slab loads by the last arriver.
#pragma once
#include "latent.hpp"
#include "kernels_aux.hpp"

namespace vaeb {

// [dMu | dLv] of element (m, j) from dzsum = sum_l dZ_l and dzes = sum_l dZ_l eps_l
// (LB / FV: KL direct terms; LA: the prior-logQ direct terms, VAEB.py:322-325).
DEV void latent_bwd_elem(const StepArgs& a, bool valid, int m, int j, float mu, float lv, const float* epre,
                         const float* zpre, float dzsum, float dzes, float& dmu, float& dlv) {
    const int Z = a.Z;
    const float sl = a.sc / (float)a.L;
    const float sd = fexp(0.5f * lv);
    dmu = 0.f;
    dlv = 0.f;
    if (!valid) return;
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

// One dhd tile (bx = row block of the L * Mbp decoder rows, by = H column tile) + its dZ
// slab; the last arriver of latent row block bx % (Mbp / 16) finishes the latent backward.
// red: >= 512 f32x4 of LDS (CT = 2, NWV = 16: 2048).
// HO 2 (deferred, VAEB_BWD_DEFER): the tile stores its slab plainly and ends; the last
// launch's reducer workgroups sum the slabs (kernels_aux.hpp LatRed).
// AT (atomic hand-off, latent.hpp fx_*): instead of a dZ slab, the tile adds its partial
// dZ_l(m, j) into S(m, j) = sum_l dZ_l and dZ_l eps_l(m, j) into E(m, j) = sum_l dZ_l eps_l
// (acc_dz; L * ceil(H / 16 CT) contributors each); the add completing S stores dMu(m, j), the
// one completing E stores dLv(m, j).  dZ itself is not stored on this path.
// CT column tiles per workgroup over NWV waves splitting K (CT = 2, NWV = 16: 1024-thread
// workgroups, the encoder's enc_latent16 geometry): half the contributors per latent element,
// so MNIST 784-500-20 (32 H column tiles) comes under the counted atomics' fan-in limit of 16
// and the latent backward completes inside this launch -- the last launch then starts from a
// finished [dMu | dLv] instead of reducing slabs and handing them to its tiles in-launch.
template <bool V>
struct PDhdCT : PDhdT<V> {
    DEV f32x4 b4(int n, int k, int w) const { return this->ld(this->bw, this->wplane, n + 16 * w, this->a.H, k); }
};
template <int NCT, int GCH, bool V, int HO, int CT = 1, int NWV = 8>
DEV void dhd_dz_body(const PDhdT<V>& p0, int bx, int by, f32x4* red, int sid) {
    static_assert(CT == 1 || (HO == 1 && NWV == 16), "two column tiles: the atomic hand-off on 16 waves");
    constexpr bool AT = HO == 1;
    constexpr int NTH = 64 * NWV;
    constexpr int NS = NWV == 16 ? 1 : NCT;   // atomic-add slots per thread: 32 Z <= 1024
    __shared__ float ts[16][16 * CT + 4];
    __shared__ int sflag;
    __shared__ float pm[AT ? 64 : 1][17];   // AT: [dZ | dZ eps] partials, [column][row]
    PDhdCT<V> p{p0};
    p.prepare();
    const StepArgs& a = p.a;
    VAEB_STAMP_AT(a, sid, 0);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, q = lane >> 4;
    const int Z = a.Z, H = a.H;
    const int m0 = bx * 16, n0 = by * 16 * CT;
    const int nrb = a.Mbp >> 4, nctH = (H + 16 * CT - 1) / (16 * CT);
    const int l = bx / nrb, rbl = bx % nrb;

    // Row-parallel epilogue: phase A -- wave w < 4 CT finishes row group r = w & 3 of column
    // tile w >> 2 (sum of the NWV K-slice partials, dtanh, dA1); phase B -- wave ct < NCT forms
    // the tile's partial dZ for latent tile ct from all of dA1 through LDS (one wave running
    // both phases serially took ~1.3 us of the launch's critical path).
    const int er = wave & 3, ca = wave >> 2;
    float hdv = 0.f;
    f32x4 w1v[CT];
    float ev[4];   // HO: eps_l at (row 4q + r, latent j = 16 wave + li)
    if (wave < 4 * CT) {
        const int n = n0 + 16 * ca + li, m = m0 + 4 * q + er;
        hdv = bld(mkbuf(a.hd, (int64_t)a.Me * H * 4), (n < H && m < a.Me) ? (uint32_t)(m * H + n) * 4u : kOOB);
    }
    if (wave < NCT) {
        // W1^T rows n0 + 16 c .. + 15 at latent j = 16 wave + li: 4 consecutive n per lane
        const rsrc_t bw1 = mkbuf(a.W1, (int64_t)Z * H * 4);
        const bool vh = (H & 3) == 0 && aligned16(a.W1);
#pragma unroll
        for (int c = 0; c < CT; ++c) w1v[c] = kc4(bw1, H, wave * 16 + li, n0 + 16 * c + 4 * q, Z, H, vh);
        if constexpr (AT) {
            const rsrc_t be = mkbuf(a.eps, (int64_t)a.Me * Z * 4);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = wave * 16 + li, m = rbl * 16 + 4 * q + r;
                ev[r] = bld(be, j < Z ? (uint32_t)((l * a.Mbp + m) * Z + j) * 4u : kOOB);
            }
        }
    }
    // AT: mu, lv of each element this thread may complete (column c: dMu | dLv of latent c % Z)
    float muv[NS], lvv[NS];
    if constexpr (AT) {
        const rsrc_t bm = mkbuf(a.mu, (int64_t)a.Mbp * Z * 4), bl = mkbuf(a.lv, (int64_t)a.Mbp * Z * 4);
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            const int e = (int)threadIdx.x + NTH * u, c = e >> 4, m = rbl * 16 + (e & 15);
            const uint32_t o = e < 32 * Z ? (uint32_t)(m * Z + (c < Z ? c : c - Z)) * 4u : kOOB;
            muv[u] = bld(bm, o);
            lvv[u] = bld(bl, o);
        }
    }
    f32x4 acc[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[c] = zero4();
    wave_mainloop<CT, NWV, GCH>(p, m0 + li, n0 + li, p.K, wave, acc);
    VAEB_STAMP_AT(a, sid, 1);
    float* redf = reinterpret_cast<float*>(red);   // [c][r][slice][lane]
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) redf[((c * 4 + r) * NWV + wave) * 64 + lane] = acc[c][r];
    __syncthreads();
    if (wave < 4 * CT) {
        float t = redf[((ca * 4 + er) * NWV) * 64 + lane];
#pragma unroll
        for (int sl = 1; sl < NWV; ++sl) t += redf[((ca * 4 + er) * NWV + sl) * 64 + lane];
        const int n = n0 + 16 * ca + li, m = m0 + 4 * q + er;
        const float v = (n < H && (m % a.Mbp) < a.Mb) ? t * (1.f - hdv * hdv) : 0.f;
        if (n < H) a.dA1[(int64_t)m * H + n] = v;
        ts[4 * q + er][16 * ca + li] = v;
    }
    __syncthreads();
    if (wave < NCT) {
        // partial dZ of this tile, latent tile ct = wave: (16 x 16 CT dA1) . (16 CT rows of W1^T)
        f32x4 sv = zero4();
#pragma unroll
        for (int c = 0; c < CT; ++c) {
            f32x4 av;
#pragma unroll
            for (int s = 0; s < 4; ++s) av[s] = ts[li][16 * c + 4 * q + s];
            sv = mfma4(av, w1v[c], sv);
        }
        const int j = wave * 16 + li;
        if constexpr (AT) {
            if (j < Z)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    pm[j][4 * q + r] = sv[r];
                    pm[Z + j][4 * q + r] = sv[r] * ev[r];
                }
        } else {
            const rsrc_t bs = mkbuf(a.slab_dz, (int64_t)a.L * a.Mbp * nctH * Z * 4);
            const int64_t blk = ((int64_t)l * nrb + rbl) * nctH + by;
            const uint32_t so = j < Z ? (uint32_t)(((blk * Z + j) * 16 + 4 * q) * 4) : kOOB;
            // HO 2 (deferred): plain stores, published by the kernel boundary to the reducers
            // of the last launch (kernels_aux.hpp LatRed); HO 0: write-through for the ticket
            if constexpr (HO == 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, sv), bs, so, 0, 0);
            else st4_sc1(bs, so, sv);
        }
    }
    if constexpr (AT) {
        // column c < Z: S = sum_l dZ_l of latent c; c >= Z: E = sum_l dZ_l eps_l of latent c - Z
        __syncthreads();
        VAEB_STAMP_AT(a, sid, 4);   // (timeline build: the partials are in LDS)
        FxSlots<NS, NTH> fx;
        fx.add(a.acc_dz, a.acc_ml - 1, rbl * 16, 2 * Z, pm, 32 * Z);   // guard: blk[kBlkFxErr]
        if (VAEB_DBG_ON(a.dbg)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        VAEB_STAMP_AT(a, sid, 3);   // (timeline build: this thread's adds returned)
        const float sl = a.sc / (float)a.L;
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            float v;
            if (!(fx.ok[u] && fx_done(fx.t[u], nctH * a.L, v))) continue;
            const int c = fx.col[u], m = rbl * 16 + fx.row[u];
            const bool isE = c >= Z;
            const int j = isE ? c - Z : c;
            const bool valid = m < a.Mb;
            const float mu = muv[u], lv = lvv[u], sd = fexp(0.5f * lv);
            float tm = 0.f, tv = 0.f;
            if (a.est == EST_LA && valid) {
                for (int s = 0; s < a.L; ++s) {
                    const int64_t os = ((int64_t)s * a.Mbp + m) * Z + j;
                    const float zs = a.z[os];
                    tm += -zs;
                    tv += 0.5f - 0.5f * zs * sd * a.eps[os];
                }
            }
            float d;
            if (!isE) d = a.est == EST_LA ? v + sl * tm : v - a.sc * mu;
            else d = a.est == EST_LA ? v * 0.5f * sd + sl * tv : v * 0.5f * sd + a.sc * 0.5f * (1.f - fexp(lv));
            a.dMuLv[(int64_t)m * 2 * Z + c] = valid ? d : 0.f;
            fx_reset(fx_at(a.acc_dz, (int64_t)m * 2 * Z + c));
        }
        VAEB_STAMP_AT(a, sid, 2);
        return;
    }
    VAEB_STAMP_AT(a, sid, 2);
    if constexpr (HO == 2) {
        // the last launch's reducers count their arrivals on the counter replicas cnt_dz[16 c]
        // (kernels_aux.hpp kLatCnt; zeroed here, before it)
        if (sid == 0 && (int)threadIdx.x < kLatCnt) a.cnt_dz[threadIdx.x * kLatCntStride] = 0;
        return;
    }
    if (!arrive_last<NCT>(a.cnt_dz + rbl, nctH * a.L, &sflag)) return;
    VAEB_STAMP_AT(a, sid, 3);

    // ---- reducer: latent row block rbl, all L planes.  Thread (ml, j) owns one element;
    // its element-wise operands ride the round trip of the first slab loads.
    const int ml = threadIdx.x >> 5, j = threadIdx.x & 31;
    const int m = rbl * 16 + ml;
    const bool valid = j < Z && m < a.Mb;
    const uint32_t oj = valid ? (uint32_t)(m * Z + j) * 4u : kOOB;
    const float mu = bld(mkbuf(a.mu, (int64_t)a.Mbp * Z * 4), oj);
    const float lv = bld(mkbuf(a.lv, (int64_t)a.Mbp * Z * 4), oj);
    float epre[kLP], zpre[kLP];
    {
        const rsrc_t be = mkbuf(a.eps, (int64_t)a.Me * Z * 4);
        const rsrc_t bz = mkbuf(a.z, (int64_t)a.Me * Z * 4);
#pragma unroll
        for (int s = 0; s < kLP; ++s) {
            const uint32_t o = (valid && s < a.L) ? (uint32_t)((s * a.Mbp + m) * Z + j) * 4u : kOOB;
            epre[s] = bld(be, o);
            zpre[s] = (a.est == EST_LA) ? bld(bz, o) : 0.f;
        }
    }
    const rsrc_t bs = mkbuf(a.slab_dz, (int64_t)a.L * a.Mbp * nctH * Z * 4);
    const int NF4 = 4 * Z;            // float4 per slab (Z columns x 16 rows)
    const int NP = 512 / NF4;         // slab partitions (threads >= NP * NF4 idle)
    const int f = threadIdx.x % NF4, part = threadIdx.x / NF4;
    float dzsum = 0.f, dzes = 0.f;
    for (int s = 0; s < a.L; ++s) {
        const int64_t first = ((int64_t)s * nrb + rbl) * nctH * NF4;
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
        float dz = 0.f;
        if (j < Z) {
            const int ff = (j * 16 + ml) >> 2, comp = ml & 3;
            for (int pp = 0; pp < NP; ++pp) dz += red[pp * NF4 + ff][comp];
        }
        dz = valid ? dz : 0.f;
        const float e = (s < kLP) ? epre[s] : (valid ? a.eps[((int64_t)s * a.Mbp + m) * Z + j] : 0.f);
        dzsum += dz;
        dzes += dz * e;
        if (j < Z) a.dZ[((int64_t)s * a.Mbp + m) * Z + j] = dz;
        __syncthreads();
    }
    VAEB_STAMP_AT(a, sid, 4);
    if (j < Z) {
        float dmu, dlv;
        latent_bwd_elem(a, valid, m, j, mu, lv, epre, zpre, dzsum, dzes, dmu, dlv);
        a.dMuLv[(int64_t)m * 2 * Z + j] = dmu;
        a.dMuLv[(int64_t)m * 2 * Z + Z + j] = dlv;
    }
    VAEB_STAMP_AT(a, sid, 5);
}

// Side duties of the dhd launch.  pend (the deferred dW2: no dW2 tiles in this grid): set to 1
// -- the next step's encoder launch, or the host's flush, runs this step's dW2 (| dW6)
// (latent.hpp enc_latent16_w2_kernel).
struct DhdAux {
    int* pend;
};

// dhd (+ dZ slabs, latent backward) tiles and the dW2 (| dW6) weight-gradient tiles in one
// grid.  The dhd tiles are dispatched first: with the latent backward behind them they are
// the launch's critical path (tile_wgrad_kernel, without it, puts the dW2 blocks first).
template <int NCT, int GCH, bool VEC, int TS, int HO>
// aux: side duties of the dhd launch (DhdAux)
__global__ __launch_bounds__(512) void dhd_dz_wgrad_kernel(PDhdT<VEC> p, WGradArgs w, int ntile, int gx, DhdAux aux) {
    __shared__ float sa[kWKB][kWP];
    __shared__ float sb[kWKB][kWP];
    const int nwg = w.total_wgs - ntile;   // grid = w.total_wgs (no implicit-argument load)
    const int b0 = blockIdx.x;
    if (aux.pend && b0 == 0 && threadIdx.x == 0) *aux.pend = 1;
    const int bid = b0 < ntile ? xcd_remap(b0, ntile) : ntile + xcd_remap(b0 - ntile, nwg);
    if (bid < ntile) {
        dhd_dz_body<NCT, GCH, VEC, HO>(p, bid % gx, bid / gx, reinterpret_cast<f32x4*>(&sa[0][0]), bid);
        return;
    }
    if (VAEB_DBG_ON(w.dbg) && threadIdx.x == 0) w.dbg[bid * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    wgrad_body<VEC, 8, TS>(w, w.g[0], bid, sa, sb);
}

}  // namespace vaeb
