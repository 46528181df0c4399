// thin_bf16.hpp -- the latent-width products of the bf16 step with the latent block fused
// into their epilogues (config 5: B = 8192, H = 2048, Z = 128).
//
//   heads + latent forward:  [mu | lv] = h [W4 | W5] + [b4 | b5]   (VAEB.py:248-249)
//                            eps, z = mu + exp(lv / 2) eps, KL terms (VAEB.py:41-47, 343)
//   dz + latent backward:    dZ = dA1 W1^T,  [dMu | dLv], b4 / b5 column sums
//
// On the 256-row GEMM engine these products (N = 2Z = 256 or Z = 128 output columns) had
// too few tiles to fill the chip, so they ran split-K and handed fp32 slabs to a latent
// kernel: at config 5 the heads slabs alone were 64 MB written and read back (heads +
// latent 29 us, dz + latent_bwd 23 us, both HBM-bound on slab traffic).  Here a block owns
// BMT rows x 128 output columns over the FULL K, so the result never leaves registers: the
// latent element-wise work runs on the accumulators and only mu / lv / eps / z (or
// [dMu | dLv]) are written.  Measured at config 5 (scripts/gpu_r3_bfab.sh, VAEB_BF_THIN):
// heads + latent 28.6 -> 28.9 us (each block streams 256 KiB of h and re-reads 512 KiB of
// [W4 | W5] from L2: ~26 KiB/us per CU, the per-CU operand ingest, not the slabs, bounds
// it), dz + latent backward 23.6 -> 20.5 us, step 792 -> 785 / 786 -> 778 us in alternating
// runs.  256 blocks at config 5, one per CU:
//   * heads: BMT = 64 rows x (64 latents of mu | the same 64 of lv) -- the two halves of
//     the tile are the two column ranges [j0, j0 + 64) and [Z + j0, Z + j0 + 64) of the
//     K-outer [W4 | W5] shadow, so every lane holds mu and lv of the same element;
//   * dz: BMT = 32 rows x 128 latents of the K-contiguous W1 shadow.
// Operands reach LDS by LDS-DMA into a 3-stage ring (prefetch distance 2) in the GEMM
// engine's image formats (gemm_bf16.hpp: swizzled KC / KO images of BK = 32 k, read with
// frag<>); a stage holds KT K-tiles so that every wave issues the same number of 1-KiB
// pieces (BMT 64: KT 2, 3 pieces per wave; BMT 32: KT 4, 5 per wave), which the counted
// vmcnt waits rely on.  Eight waves: wave (wr, wc) owns the 16-row block wr and TPW
// 16-column MFMA tiles of column group wc.
// Included twice by h16_engines.hpp (namespace VAEB_H16NS = bf / hf), after step_bf16.hpp.

namespace vaeb {
namespace VAEB_H16NS {

template <int BMT>
struct ThinShape {
    static constexpr int NT = 128;                  // output columns per block
    static constexpr int RBK = BMT / 16;            // 16-row blocks
    static constexpr int CG = NWAVE / RBK;          // column groups of waves
    static constexpr int TPW = NT / 16 / CG;        // MFMA tiles per wave
    static constexpr int kA = BMT * BK * 2;         // KC image of one K-tile of A
    static constexpr int kB = BK * NT * 2;          // image of one K-tile of B
    static constexpr int KT = BMT == 64 ? 2 : 4;    // K-tiles per stage
    static constexpr int kPA = KT * kA / 1024, kPB = KT * kB / 1024;   // 1-KiB pieces
    static constexpr int kPerWave = (kPA + kPB) / NWAVE;
    static_assert((kPA + kPB) % NWAVE == 0 && kA % 1024 == 0, "thin: pieces per wave");
    static constexpr int kStage = KT * (kA + kB);
    // 3-stage ring (prefetch distance 2); 6 x 24 KiB / 4 x 40 KiB rings measured slower
    // (heads 28.9 -> 32.2 us, dz 20.5 -> 21.4): the stream is throughput-, not latency-bound
// heads (BMT 64): 4 stages of 24 KiB (round 5: 31.2 -> 28.4 us against 3; 6 stages 32.4)
    static constexpr int kStages = BMT == 64 ? 4 : 3;
    static constexpr int kSmem = kStages * kStage;
};

struct ThinArgs {
    const bf16_t* A; int lda; int64_t a_bytes; int M;   // A: [M][K] (K-contiguous)
    const bf16_t* B; int ldb; int64_t b_bytes;           // B: KO [K][ldb] or KC [N][ldb]
    int K;
    int bcol1;   // KO with a split column map: image columns 64.. map to bcol1 + (c - 64)
};

template <int N>
DEV void thin_wait() {   // all but the N youngest vector-memory ops done, LDS ops done; barrier
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
// wait for the oldest stage in flight when `after` younger stages (of P pieces each) are
template <int P>
DEV void thin_wait_after(int after) {
    switch (after) {
        case 0: thin_wait<0>(); break;
        case 1: thin_wait<P>(); break;
        case 2: thin_wait<2 * P>(); break;
        case 3: thin_wait<3 * P>(); break;
        case 4: thin_wait<4 * P>(); break;
        default: thin_wait<5 * P>(); break;
    }
}

// Block (bm = row block, bn = column block) of C = A B; epilogue e(acc, m0, bn, wr, wc).
template <int LB, int BMT, class Epi>
DEV void thin_body(const ThinArgs& t, const Epi& e, int bm, int bn, char* smem) {
    using S = ThinShape<BMT>;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave % S::RBK, wc = wave / S::RBK;
    const int m0 = bm * BMT;
    const v4i da = mkdesc(t.A, t.a_bytes), db = mkdesc(t.B, t.b_bytes);
    // column map of the B image: KC -- rows n = bn * 128 + c; KO -- columns j0 + c (c < 64)
    // and bcol1 + c - 64 (c >= 64) when bcol1 >= 0, else bn * 128 + c
    const int j0 = bn * (t.bcol1 >= 0 ? 64 : S::NT);
    typename Epi::Pre pre = e.prefetch(m0, bn, wr, wc, lane);

    const int nst = (t.K + S::KT * BK - 1) / (S::KT * BK);
    constexpr int rot = 0;
    auto issue = [&](int st_) {   // ring stage st_: K-tiles kt = st * KT + u of stage st = (st_ + rot) mod nst
        char* img = smem + (st_ % S::kStages) * S::kStage;
        const int st = st_ + rot < nst ? st_ + rot : st_ + rot - nst;
#pragma unroll
        for (int i = 0; i < S::kPerWave; ++i) {
            const int piece = wave * S::kPerWave + i;
            uint32_t off, lds;
            if (piece < S::kPA) {   // A: KC image [BMT rows][32 k], 64-B rows
                constexpr int PPI = S::kA / 1024;
                const int u = piece / PPI, byte = (piece % PPI) * 1024 + lane * 16;
                const int row = byte >> 6, p = (byte >> 4) & 3;
                const int k = (st * S::KT + u) * BK + (p ^ swz_kc(row)) * 8, r = m0 + row;
                off = (r < t.M && k < t.K) ? ((uint32_t)r * (uint32_t)t.lda + (uint32_t)k) * 2u : kOOB;
                lds = (uint32_t)(uintptr_t)(img + u * S::kA + (piece % PPI) * 1024);
            } else {
                constexpr int PPI = S::kB / 1024;
                const int pb0 = piece - S::kPA;
                const int u = pb0 / PPI, byte = (pb0 % PPI) * 1024 + lane * 16;
                const int kt0 = (st * S::KT + u) * BK;
                if constexpr (LB == KC) {   // [128 rows n][32 k]
                    const int row = byte >> 6, p = (byte >> 4) & 3;
                    const int k = kt0 + (p ^ swz_kc(row)) * 8, n = bn * S::NT + row;
                    off = (k < t.K) ? ((uint32_t)n * (uint32_t)t.ldb + (uint32_t)k) * 2u : kOOB;
                } else {                    // [32 k-rows][128 columns], 256-B k-rows
                    const int kr = byte >> 8, p = (byte >> 4) & 15;
                    const int c = 8 * (p ^ swz_ko(kr));
                    const int col = t.bcol1 >= 0 ? (c < 64 ? j0 + c : t.bcol1 + j0 + c - 64) : j0 + c;
                    const int k = kt0 + kr;
                    off = (k < t.K) ? ((uint32_t)k * (uint32_t)t.ldb + (uint32_t)col) * 2u : kOOB;
                }
                lds = (uint32_t)(uintptr_t)(img + S::KT * S::kA + u * S::kB + (pb0 % PPI) * 1024);
            }
            dma16(piece < S::kPA ? da : db, off, __builtin_amdgcn_readfirstlane(lds));
        }
    };

    f32x4 acc[S::TPW];
#pragma unroll
    for (int j = 0; j < S::TPW; ++j) acc[j] = zero4();
    // prefetch distance.  heads (4 stages): kStages - 2, so a stage is refilled two iterations
    // after its last read, behind the next iteration's wait barrier, and the barrier at the end of
    // each stage is not needed (heads 28.5 -> 27.1 us; 5 stages that way 30.4); dz: kStages - 1
    constexpr bool k1Bar = BMT == 64;
    constexpr int PD = k1Bar ? S::kStages - 2 : S::kStages - 1;
    static_assert(PD <= 5, "thin_wait_after");
    for (int st = 0; st < PD && st < nst; ++st) issue(st);
    for (int st = 0; st < nst; ++st) {
        if (st + PD < nst) issue(st + PD);
        thin_wait_after<S::kPerWave>(min(nst - 1, st + PD) - st);
        const char* img = smem + (st % S::kStages) * S::kStage;
#pragma unroll
        for (int u = 0; u < S::KT; ++u) {
            const char* As = img + u * S::kA;
            const char* Bs = img + S::KT * S::kA + u * S::kB;
            const bf16x8 af = frag<KC, BMT>(As, 16 * wr, 0, lane);
            bf16x8 bfr[S::TPW];
#pragma unroll
            for (int j = 0; j < S::TPW; ++j) bfr[j] = frag<LB, S::NT>(Bs, Epi::col(wc, j), 0, lane);
#pragma unroll
            for (int j = 0; j < S::TPW; ++j) acc[j] = mfma16(af, bfr[j], acc[j]);
        }
        if constexpr (!k1Bar) {
            __builtin_amdgcn_s_barrier();   // stage st's buffer is refilled by the issue of st + kStages
            asm volatile("" ::: "memory");
        }
    }
    e.apply(acc, pre, m0, bn, wr, wc, lane);
}

template <int LB, int BMT, class Epi>
__global__ __launch_bounds__(NTHR, 2) void thin_kernel(ThinArgs t, Epi e) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    thin_body<LB, BMT, Epi>(t, e, blockIdx.x, blockIdx.y, smem);
}

// ---- heads + latent forward (BMT 64, TPW 4: tiles 0, 1 = mu, 2, 3 = lv of latents
// j0 + 32 wc + 16 {0, 1} + (lane & 15)).  Same outputs as latent_fwd_v4_kernel (LB, L = 1):
// mu, lv, eps, z (bf16), and per row one KL partial per 64-latent column block
// (kl_part[m * nkl + bn], summed by the ELBO reduction with the others).
struct EpiHeadsLatent {
    const float *b4, *b5;
    float *mu, *lv, *eps;
    bf16_t* z;
    float* kl_part; int nkl;
    int M, Z, mode;
    int eps_mode; uint64_t seed; const int64_t* step; uint32_t domain;
    const float* eps_in; int64_t eps_in_ld;
    BatchRef rows; int64_t row_base_mul, row_base_add;
    struct Pre { float b4[2], b5[2]; };
    DEV static int col(int wc, int j) { return j < 2 ? 32 * wc + 16 * j : 64 + 32 * wc + 16 * (j - 2); }
    DEV Pre prefetch(int, int bn, int, int wc, int lane) const {
        Pre p;
        const rsrc_t bb4 = mkbuf(b4, (int64_t)Z * 4), bb5 = mkbuf(b5, (int64_t)Z * 4);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int j = bn * 64 + 32 * wc + 16 * t + (lane & 15);
            p.b4[t] = bld(bb4, (uint32_t)j * 4u);
            p.b5[t] = bld(bb5, (uint32_t)j * 4u);
        }
        return p;
    }
    DEV void apply(const f32x4 (&acc)[4], const Pre& p, int m0, int bn, int wr, int wc, int lane) const {
        __shared__ float klw[8][16];
        const int q = lane >> 4, li = lane & 15;
        const int64_t brow = rows.order ? (int64_t)rows.order[*rows.cursor] : 0;
        const uint64_t c23 = philox_c23(*step, domain);
        float kl[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int j = bn * 64 + 32 * wc + 16 * t + li;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + 16 * wr + 4 * q + r;
                if (m >= M) continue;
                const float mv = acc[t][r] + p.b4[t], lvv = acc[t + 2][r] + p.b5[t];
                const float sd = fexp(0.5f * lvv);
                kl[r] += 0.5f * (1.f + lvv - mv * mv - fexp(lvv));
                float e = 0.f;
                if (mode != MODE_RECON) {
                    if (eps_mode == 0) e = philox_normal(seed, (uint32_t)(brow * row_base_mul + row_base_add + m), (uint32_t)j, c23);
                    else e = eps_in[(int64_t)m * Z + j];
                }
                const int64_t o = (int64_t)m * Z + j;
                mu[o] = mv;
                lv[o] = lvv;
                eps[o] = e;
                z[o] = (bf16_t)f2bf(mv + sd * e);
            }
        }
        // the row's KL over this block's 64 latents: the 16 lanes of a row group (DPP), then
        // the two column groups in order
        const int wave = threadIdx.x >> 6;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float v = sum16(kl[r]);
            if (li == 0) klw[wave][4 * q + r] = v;
        }
        __syncthreads();
        if (wc == 0 && lane < 16) {
            const int m = m0 + 16 * wr + lane;
            const float v = klw[wr][lane] + klw[wr + 4][lane];
            if (m < M) kl_part[(int64_t)m * nkl + bn] = v;
        }
    }
};

// ---- dz + latent backward (BMT 32, TPW 2: latents 32 wc + 16 {0, 1} + (lane & 15) of the
// 128-latent block bn).  Same outputs as latent_bwd_v4_kernel (LB, L = 1): [dMu | dLv] bf16
// and the 16-row-block column sums colpart[m / 16][2Z].
struct EpiDzLatent {
    const float *mu, *lv, *eps;
    bf16_t* dmulv;
    float* colpart;
    float sc;
    int M, Z;
    struct Pre { float mu[2][4], lv[2][4], e[2][4]; };
    DEV static int col(int wc, int j) { return 32 * wc + 16 * j; }
    DEV Pre prefetch(int m0, int bn, int wr, int wc, int lane) const {
        Pre p;
        const int q = lane >> 4, li = lane & 15;
        const rsrc_t bmu = mkbuf(mu, (int64_t)M * Z * 4), blv = mkbuf(lv, (int64_t)M * Z * 4),
                     bep = mkbuf(eps, (int64_t)M * Z * 4);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + 16 * wr + 4 * q + r, j = bn * 128 + 32 * wc + 16 * t + li;
                const uint32_t o = m < M ? (uint32_t)(m * Z + j) * 4u : kOOB;
                p.mu[t][r] = bld(bmu, o);
                p.lv[t][r] = bld(blv, o);
                p.e[t][r] = bld(bep, o);
            }
        return p;
    }
    DEV void apply(const f32x4 (&acc)[2], const Pre& p, int m0, int bn, int wr, int wc, int lane) const {
        const int q = lane >> 4, li = lane & 15;
        const int Z2 = 2 * Z;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int j = bn * 128 + 32 * wc + 16 * t + li;
            float cm = 0.f, cv = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + 16 * wr + 4 * q + r;
                const float dz = acc[t][r];
                const float sd = fexp(0.5f * p.lv[t][r]);
                const float dm = dz - sc * p.mu[t][r];
                const float dl = dz * 0.5f * sd * p.e[t][r] + sc * 0.5f * (1.f - fexp(p.lv[t][r]));
                if (m < M) {
                    dmulv[(int64_t)m * Z2 + j] = (bf16_t)f2bf(dm);
                    dmulv[(int64_t)m * Z2 + Z + j] = (bf16_t)f2bf(dl);
                    cm += dm;
                    cv += dl;
                }
            }
            // the 16-row block's column sums: the 4 row groups of the column (lanes li + 16 q)
            cm += __shfl_xor(cm, 16, 64);
            cm += __shfl_xor(cm, 32, 64);
            cv += __shfl_xor(cv, 16, 64);
            cv += __shfl_xor(cv, 32, 64);
            const int rb = (m0 >> 4) + wr;
            if (q == 0 && 16 * rb < M) {
                colpart[(int64_t)rb * Z2 + j] = cm;
                colpart[(int64_t)rb * Z2 + Z + j] = cv;
            }
        }
    }
};

}  // namespace VAEB_H16NS
}  // namespace vaeb
