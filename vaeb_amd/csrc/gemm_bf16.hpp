// gemm_bf16.hpp -- bf16 MFMA GEMM engine for the large-batch SGVB step (gfx950).
//
// BASELINE config 5 (synthetic 4096 -> 2048 -> 128, batch 8192 per GPU) is a chain of
// dense contractions big enough to fill the chip, so unlike the batch-100 fp32 path
// (tile_engine.hpp, latency-bound) this engine is built for MFMA throughput:
//
//  * C[M x N] = sum_k A(m, k) B(k, n) with bf16 operands and fp32 accumulation on
//    v_mfma_f32_16x16x32_bf16 (lane l holds A[l&15][8(l>>4)+j] and B[8(l>>4)+j][l&15],
//    C/D: col = l&15, row = 4(l>>4)+r);
//  * every operand is used IN ITS NATURAL LAYOUT: an operand is either K-contiguous
//    (KC, stored [rows][K]) or K-outer (KO, stored [K][rows]).  KC tiles are read with
//    ds_read_b128, KO tiles with the gfx950 transposing read ds_read_b64_tr_b16 -- so
//    the forward (X W3), the data-gradient (dA2 W2^T) and the weight-gradient
//    (X^T dA3) products all read the same single copy of each weight / activation and
//    no transposed copies are ever written;
//  * block tile 256 x BNT x 32 (BK), 512 threads = 8 waves: BNT = 256 (waves 2 x 4,
//    128 x 64 each) or BNT = 128 for products with too few 256-wide tiles to fill the chip
//    (waves 4 x 2, 64 x 64 each); one block per CU;
//  * operand tiles reach LDS by LDS-DMA (buffer_load_dwordx4 ... lds, inline asm) into a
//    4-stage ring, prefetch distance 3, with counted s_waitcnt vmcnt(N) (never 0 inside the
//    loop); on the 256 x 256 tile waves 4-7 run one barrier behind waves 0-3 (wave-group
//    ping-pong: one reads fragments while its SIMD partner issues MFMAs);
//  * LDS images are XOR-swizzled so the fragment reads are bank-conflict free, the
//    swizzle applied to the DMA SOURCE chunk (the DMA writes each 1-KiB piece linearly):
//    KC (64-B rows): 16-B chunk c of row r at c ^ g[(r >> 2) & 3], g = {0, 2, 3, 1}
//    (ds_read_b128 lane groups of MI355X_MICROARCH.md §LDS); KO (2 BNT-byte k-rows):
//    chunk c of k-row r at c ^ (((r & 3) << 1) | (((r >> 3) & 1) << 3))
//    (ds_read_b64_tr_b16 32-lane halves);
//  * operand loads are 16-B raw buffer loads; a chunk outside [0, rows) x [0, K) is
//    redirected out of range and reads 0 (tails need rows and K to be multiples of 8);
//  * split-K over gridDim.y for the thin products (latent-width N or M): each slice
//    stores an fp32 slab that a later kernel sums in fixed order (deterministic);
//  * tile order: the linear block id is remapped so that the blocks sharing one XCD
//    (blockIdx % 8, guide T1) take a contiguous run of tiles, grouped 8 row tiles at a
//    time so concurrently running blocks share operand panels in that XCD's L2.
// Epilogues are functors applied to the wave's accumulator block (128 x 64 or 64 x 64) in
// registers.
//
// Included twice by h16_engines.hpp: namespace VAEB_H16NS = bf with VAEB_H16_F16 = 0 (bf16
// operands, v_mfma_f32_16x16x32_bf16) and VAEB_H16NS = hf with VAEB_H16_F16 = 1 (fp16 operands,
// v_mfma_f32_16x16x32_f16, the same rate on gfx950).  Everything but the conversions and the
// MFMA below is the same code: both formats are 16 bits per element in LDS, in the transposing
// reads and in memory.  (The names bf16_t / bf16x8 / f2bf / bf2f stand for "this
// instantiation's 16-bit type".)
#include <type_traits>
#include "tile_engine.hpp"
#include "h16_common.hpp"

namespace vaeb {
namespace VAEB_H16NS {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef uint16_t bf16_t;   // raw bf16 bits in memory

enum : int { KC = 0, KO = 1 };
// Block tile BM x BNT x BK with BNT = 256 (8 waves as 2 x 4, 128 x 64 each) or 128
// (8 waves as 4 x 2, 64 x 64 each; for products with too few 256-wide tiles to fill the
// chip).  BN is the widest tile (it sizes the epilogue LDS tile).
constexpr int BM = 256, BN = 256, BK = 32, NTHR = 512, NWAVE = 8;
constexpr int kATileBytes = BM * BK * 2;         // A operand tile image (16 KiB)
template <int BNT, int ST = 4>
struct Shape {
    static constexpr int WGN = BNT / 64, WGM = NWAVE / WGN;   // wave grid
    static constexpr int TM = BM / WGM / 16, TN = 4;          // MFMA tiles per wave
    static constexpr int kB = BNT * BK * 2;                   // B operand tile image
    static constexpr int kStage = kATileBytes + kB;
    static constexpr int kPieces = (kATileBytes + kB) / 1024 / NWAVE;   // vmcnt unit per tile
    // LDS ring: 4 stages (prefetch distance 3), one block per CU; or (ST = 3, 256 x 128
    // only) 3 stages, 72 KiB with its epilogue tile, <= 128 VGPRs, two blocks per CU so
    // one block's epilogue overlaps the other's mainloop.  The weight-gradient launches
    // measured 171-183 us that way against 161-169 us with one block per CU.
    static_assert(ST == 4 || (ST == 3 && BNT == 128), "ring shape");
    static constexpr int kStages = ST;
    static constexpr int kBlocksPerCU = ST == 3 ? 2 : 1;
};

typedef float f32x2_t __attribute__((ext_vector_type(2)));
#if VAEB_H16_F16
// fp16: f32 -> fp16 round to nearest even (v_cvt_f16_f32; fp16 subnormals kept, the HIP
// default mode for 16-bit), fp16 -> f32 exact.
typedef _Float16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 bf16x2_t __attribute__((ext_vector_type(2)));
DEV uint32_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
DEV float bf2f(uint32_t b) { return (float)__builtin_bit_cast(_Float16, (uint16_t)b); }
DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
#else
// f32 -> bf16, round to nearest even: gfx950's v_cvt_pk_bf16_f32 (one instruction; the
// integer form (u + 0x7FFF + ((u >> 16) & 1)) >> 16 gives the same bits for finite inputs in
// four).  f2bf2: two values in one instruction, a in the low half.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
DEV uint32_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
DEV float bf2f(uint32_t b) { return __builtin_bit_cast(float, b << 16); }
DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
#endif
DEV uint32_t f2bf2(float a, float b) { return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t)); }
// Epilogue functors with a post(m0, n0, smem) step after store_out (kPost; gemm8_body only)
template <class E, class = void> struct HasPost : std::false_type {};
template <class E> struct HasPost<E, std::void_t<decltype(E::kPost)>> : std::bool_constant<E::kPost> {};

// KC images have 64-B rows (BK = 32): chunk c (0..3) of row r lives at c ^ g[(r >> 2) & 3],
// g = {0, 2, 3, 1}, which makes the four ds_read_b128 lane groups of a 16-row fragment read
// (MI355X_MICROARCH.md §LDS) hit 16 distinct 16-B slots.
DEV int swz_kc(int r) { return (0x78 >> (((r >> 2) & 3) * 2)) & 3; }   // g = {0, 2, 3, 1}
DEV int swz_ko(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

// One R-row x 32-k (BK) operand tile, HBM -> LDS directly (buffer_load_dwordx4 ... lds):
// each wave-instruction writes 1 KiB of the tile image linearly (lane l at byte 16 l), so
// the XOR swizzle is applied to the SOURCE chunk each lane fetches (guide rule 21): the
// lane that fills physical chunk p of a row loads logical chunk p ^ swz(row).  KC image:
// [R rows][32 k] (64-B rows); KO image: [32 k-rows][R] (2R-byte rows).  Out-of-range
// chunks are redirected past the buffer end and land as zeros.
typedef int v4i __attribute__((ext_vector_type(4)));
// Buffer descriptor as four SGPRs (base, stride 0, num_records, raw-buffer flags).
DEV v4i mkdesc(const void* p, int64_t nbytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    v4i d;
    d.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    d.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xFFFFu));
    d.z = __builtin_amdgcn_readfirstlane((int)(nbytes < 0x7FFFFFF0ll ? nbytes : 0x7FFFFFF0ll));
    d.w = 0x00020000;
    return d;
}
// One 16-B-per-lane LDS-DMA piece (buffer_load_dwordx4 ... lds) to the wave-uniform LDS
// address `lds`.  Issued from inline asm ON PURPOSE: hipcc cannot prove the MFMA loop's
// ds_reads miss the DMA'd stage and would drain the whole ring (vmcnt(0)) before every
// read; here the kernel counts the queue itself (s_waitcnt vmcnt(6) per step).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
DEV void dma16(v4i rsrc, uint32_t voff, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                 :: "v"(voff), "s"(rsrc), "s"(lds) : "memory", "m0");
}
#pragma clang diagnostic pop

template <int LAY, int R>
struct TileDma {
    v4i buf;
    int ld;        // row stride (elements) of the stored matrix
    int rlim;      // valid rows (M or N extent)
    int klim;      // end of this block's K range
    int r0;        // first row of the tile
    static constexpr int kPieces = R * BK * 2 / 1024 / NWAVE;
    DEV void issue(char* img, int k0, int wave, int lane) const {
#pragma unroll
        for (int i = 0; i < kPieces; ++i) {
            const int piece = wave * kPieces + i;             // 1-KiB piece of the image
            const int byte = piece * 1024 + lane * 16;
            uint32_t off;
            if constexpr (LAY == KC) {
                const int row = byte >> 6, p = (byte >> 4) & 3;
                const int c = p ^ swz_kc(row);
                const int r = r0 + row, k = k0 + c * 8;
                off = (r < rlim && k < klim) ? ((uint32_t)r * (uint32_t)ld + (uint32_t)k) * 2u : kOOB;
            } else {
                constexpr int RB = 2 * R;                     // image row bytes
                const int kr = byte / RB, pb = byte % RB;
                const int p = pb >> 4;
                const int c = (p & ~15) | ((p & 15) ^ swz_ko(kr));
                const int k = k0 + kr, r = r0 + c * 8;
                off = (k < klim && r < rlim) ? ((uint32_t)k * (uint32_t)ld + (uint32_t)r) * 2u : kOOB;
            }
            dma16(buf, off, __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(img + piece * 1024)));
        }
    }
};

// Fragment (8 consecutive k of one row / column) for MFMA k-step kk (k = 32 kk ...)
// of the 16 rows starting at `row` of the tile image.
template <int LAY, int R>
DEV bf16x8 frag(const char* img, int row, int kk, int lane) {
    constexpr int RB = 2 * R;   // KO image row bytes
    if constexpr (LAY == KC) {
        const int r = row + (lane & 15);
        const int c = 4 * kk + (lane >> 4);
        return *reinterpret_cast<const bf16x8*>(img + r * (BK * 2) + ((c ^ swz_kc(r)) << 4));
    } else {
        // ds_read_b64_tr_b16: lane 4q+p of each 16-lane group supplies k-row q of its
        // 4-row block, columns 4p..4p+3; lane i receives column i, k-row q in element q.
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const int kr = 32 * kk + 8 * g + q;
        const int c = (row >> 3) + (p >> 1);
        const int o = (((c & ~15) | ((c & 15) ^ swz_ko(kr))) << 4) + (p & 1) * 8;   // swz_ko(kr+4) == swz_ko(kr)
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + kr * RB + o));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (kr + 4) * RB + o));
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    }
}

using ::vaeb::h16c::BatchRef;

struct GemmArgs {
    const bf16_t* A; int lda; int64_t a_bytes;   // a_bytes: readable extent from A
    BatchRef ab;                                 // A += ab.offset() (the dataset operand)
    const bf16_t* B; int ldb; int64_t b_bytes;
    int M, N, K;
    int tiles_m, tiles_n;
    int kslice;    // K per split-K slice (multiple of BK); gridDim.y slices
    // two-slice split-K combined in the launch (gemm8_body only, gridDim.y == 2): the first
    // slice of a tile to finish stores its fp32 partial at part + tile * 65536, the second
    // adds it and runs the epilogue; ticket[tile] orders them (zero between launches)
    float* part; int* ticket;
};

// Bijective XCD-contiguous remap of the linear tile id (guide §5 template), then a
// grouped order: runs of GM row tiles sweep all column tiles.  b: the block's index within
// this product's blocks (blockIdx.x, or its offset inside a two-product grid).
DEV void tile_of(const GemmArgs& g, int b, int& tm, int& tn) {
    constexpr int GM = 8;
    const int nwg = g.tiles_m * g.tiles_n;
    int t = b;
    if (nwg >= 16) {
        const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
        t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    }
    const int per_group = GM * g.tiles_n;
    const int grp = t / per_group, in = t - grp * per_group;
    const int gm = min(GM, g.tiles_m - grp * GM);
    tm = grp * GM + in % gm;
    tn = in / gm;
}

template <int P>
DEV void ring_wait(int after) {   // wait for all but `after` tiles' worth of LDS-DMA pieces
    if constexpr (P == 4) {
        if (after >= 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else if (after == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    } else {
        static_assert(P == 3, "ring piece count");
        if (after >= 2) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
        else if (after == 1) asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// One block tile (block `bid` of the product, K slice kz) of C = A B with epilogue e.
template <int LA, int LB, int BNT, class Epi, int ST = 4>
DEV void gemm_body(const GemmArgs& g, const Epi& e, int bid, int kz, char* smem) {
    using S = Shape<BNT, ST>;
    constexpr int TM = S::TM, TN = S::TN;
    int tm, tn;
    tile_of(g, bid, tm, tn);
    const int m0 = tm * BM, n0 = tn * BNT;
    const int kbeg = kz * g.kslice;
    const int kend = min(g.K, kbeg + g.kslice);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / S::WGN, wn = wave % S::WGN;

    const TileDma<LA, BM> la{mkdesc(g.A + g.ab.offset(), g.a_bytes), g.lda, g.M, kend, m0};
    const TileDma<LB, BNT> lb{mkdesc(g.B, g.b_bytes), g.ldb, g.N, kend, n0};

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = zero4();

    const int nkt = (kend - kbeg + BK - 1) / BK;
    auto stage = [&](int s) { return smem + s * S::kStage; };
    auto issue = [&](int t) {
        char* st = stage(t % S::kStages);
        la.issue(st, kbeg + t * BK, wave, lane);
        lb.issue(st + kATileBytes, kbeg + t * BK, wave, lane);
    };
    // Ring of 4 LDS stages, prefetch distance 3: tiles t+1..t+3 stream in while tile t is
    // multiplied.  Each wave waits only for its own pieces of tile t + 1 (counted vmcnt:
    // the pieces of the tiles issued after it stay in flight) before a barrier, and a stage
    // is read only after the barrier that follows that wait (guide §5, "Read a staged
    // buffer one phase AFTER the wait that retires it").  Raw s_barrier: __syncthreads()
    // would drain every LDS-DMA (vmcnt(0)); sched_barrier keeps hipcc from moving MFMAs
    // across the barriers.
    //
    // 256-wide tiles (PP): two wave groups in ping-pong (guide §5 "256² 8-phase
    // template": its staggered wave rows).  Group g = wave >> 2 puts one wave of each group
    // on every SIMD; group 1 runs one barrier behind group 0, so in every barrier interval
    // one group reads its fragments from LDS while the other issues its MFMAs, and each
    // SIMD's MFMA pipe alternates between its two waves.  Iteration t of a wave:
    //   R: issue the DMA of tile t + 3; ds_read tile t's fragments; wait for its own
    //      pieces of tile t + 1 and for its reads;  barrier;  M: MFMAs;  barrier.
    // Ordering (barrier numbers #k; group 0's R(t) lies between #2t and #2t + 1, group 1's
    // between #2t + 1 and #2t + 2): tile t + 1 is certified by both groups before #2t + 2,
    // ahead of every read of it; tile t - 1's stage, refilled by the DMA of tile t + 3
    // after #2t, was last read before #2t.
    // 256 x 128 tiles (64 x 64 per wave, 16 MFMAs per K-tile) measured 10-40 % slower with
    // the ping-pong, so there all waves run R, M, then certify tile t + 1 and barrier once.
    constexpr bool PP = BNT == 256;
    constexpr int PD = S::kStages - 1;   // prefetch distance
    const int grp = wave >> 2;
    for (int t = 0; t < PD && t < nkt; ++t) issue(t);
    ring_wait<S::kPieces>(min(nkt, PD) - 1);   // tile 0 certified
    __builtin_amdgcn_sched_barrier(0);
    if (PP && grp == 1) {
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    }
    for (int t = 0; t < nkt; ++t) {
        if (t + PD < nkt) issue(t + PD);
        const char* As = stage(t % S::kStages);
        const char* Bs = As + kATileBytes;
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag<LA, BM>(As, wm * (16 * TM) + 16 * i, 0, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag<LB, BNT>(Bs, wn * (16 * TN) + 16 * j, 0, lane);
        if constexpr (PP) {
            ring_wait<S::kPieces>(max(0, min(nkt - 1, t + PD) - (t + 1)));
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_setprio(1);   // keeps the MFMA cluster between the barriers (guide T5)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        if constexpr (PP) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
        } else {
            ring_wait<S::kPieces>(max(0, min(nkt - 1, t + PD) - (t + 1)));
        }
    }
    if (PP && grp == 0) __builtin_amdgcn_s_barrier();   // re-align the groups' barrier counts
    // Epilogue.  The LDS is free again (the loop ended on a barrier with nothing in
    // flight): epilogues with a bf16 input tile (x, h, hd at the output positions) fetch
    // it with coalesced 16-B loads into a padded LDS tile; bf16 results go back through the
    // same tile and leave with 16-B stores.  Waves hand 64 x 64 blocks to the epilogue.
    if constexpr (Epi::kIn) {
        e.template load_in<BNT>(m0, n0, smem);
        __syncthreads();
    }
    const int mw = m0 + wm * (16 * TM), nw = n0 + wn * (16 * TN);
    if constexpr (TM == 4) {
        e.template apply<BNT>(mw, nw, acc, kz, smem);
    } else {
        f32x4 lo[4][4], hi[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) { lo[i][j] = acc[i][j]; hi[i][j] = acc[i + 4][j]; }
        e.template apply<BNT>(mw, nw, lo, kz, smem);
        e.template apply<BNT>(mw + 64, nw, hi, kz, smem);
    }
    if constexpr (Epi::kOut) {
        __syncthreads();
        e.template store_out<BNT>(m0, n0, smem);
    }
}

template <int LA, int LB, int BNT, class Epi, int ST = 4>
__global__ __launch_bounds__(NTHR, (2 * Shape<BNT, ST>::kBlocksPerCU)) void gemm_kernel(GemmArgs g, Epi e) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    gemm_body<LA, LB, BNT, Epi, ST>(g, e, blockIdx.x, blockIdx.y, smem);
}

// Two independent products in one grid (no split-K): blocks [0, nb1) run product 1, the
// rest product 2.  Used where a product with too few 256 x 256 tiles to fill the chip
// (the weight gradient dW2 | dW6: 128 tiles at config 5, each twice as deep as the other
// product's) can share the launch with a product that needs only the same inputs (dhd:
// 256 tiles): product 1's blocks are dispatched first and each CU then holds one product-1
// tile or two product-2 tiles in sequence (config 5: 270 us against 112 + 174 us as two
// launches).  Measured and rejected: product 1 as a two-slice split-K combined in the
// launch (slice-1 blocks waiting on a flag for their slice-0 partner's fp32 partial) --
// 299 us, and dW3 the same way 169 vs 160 us: the partial slabs' write-through traffic
// and the longer epilogue tail cost more than the balanced grid saved.
template <int LA1, int LB1, class E1, int LA2, int LB2, class E2, int BNT>
__global__ __launch_bounds__(NTHR, 2 * Shape<BNT>::kBlocksPerCU) void gemm2_kernel(GemmArgs g1, E1 e1, GemmArgs g2,
                                                                                  E2 e2, int nb1) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int b = blockIdx.x;
    if (b < nb1) gemm_body<LA1, LB1, BNT, E1>(g1, e1, b, 0, smem);
    else gemm_body<LA2, LB2, BNT, E2>(g2, e2, b - nb1, 0, smem);
}

// ------------------------------------------------------------------ helpers
// Lane l's element (i, j, r) of a wave block at (mw, nw): row mw + 16i + 4(l>>4) + r,
// column nw + CM::off(j) + (l&15).  The column map CM says where the wave's four 16-column
// fragment tiles sit: ColStd -- 64 contiguous columns (gemm_body); Col8 -- two 32-column
// pieces 128 apart (gemm8_body: a wave's column quadrants of the 256-wide tile).  slot(nw):
// the per-row partial slot of the wave block (EpiDecOut), one per 64 columns of a tile.
struct ColStd {
    static constexpr int off(int j) { return 16 * j; }
    DEV static int slot(int nw) { return nw >> 6; }
};
struct Col8 {
    static constexpr int off(int j) { return 16 * (j & 1) + 128 * (j >> 1); }
    DEV static int slot(int nw) { return ((nw >> 8) << 2) + ((nw & 255) >> 5); }
};
DEV int erow(int mw, int i, int r, int lane) { return mw + 16 * i + 4 * (lane >> 4) + r; }
template <class CM = ColStd> DEV int ecol(int nw, int j, int lane) { return nw + CM::off(j) + (lane & 15); }

// Column sums of the wave's 64 x 64 block (each lane: its column of tile j), reduced
// over the 4 lane groups that share a column.  Lanes 0..15 hold the result for tile j.
DEV float colsum_lanes(float s) {
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    return s;
}

// ------------------------------------------------------------------ epilogue tiles
// A BM x W bf16 tile in LDS (W = the block's tile width) with a 2W + 32-byte row pitch
// (544 or 288 B, 8 (mod 32) dwords): the four 16-lane groups of a per-element access
// (rows 4(l>>4)+r, 16 consecutive columns) land on disjoint banks.
template <int W> constexpr int epitch() { return W * 2 + 32; }
template <int BNT, int ST = 4>
constexpr int lds_bytes() {
    constexpr int ring = Shape<BNT, ST>::kStages * Shape<BNT, ST>::kStage, epi = BM * epitch<BNT>();
    return ring > epi ? ring : epi;   // 128 KiB / 136 KiB at 256 wide, 72 KiB at 128
}
template <int W> DEV int eoff(int row, int col) { return row * epitch<W>() + col * 2; }
template <int W> DEV float lds_bf(const char* t, int row, int col) {
    return bf2f(*reinterpret_cast<const uint16_t*>(t + eoff<W>(row, col)));
}
template <int W> DEV void lds_st_bf(char* t, int row, int col, float v) {
    *reinterpret_cast<uint16_t*>(t + eoff<W>(row, col)) = (uint16_t)f2bf(v);
}
// Cooperative tile copies: rows [0, BM) x columns [0, CW) of the tile at (r0, c0) of a
// [rows x ld] bf16 matrix into / out of the W-wide LDS tile; rows >= rlim or columns >=
// clim read 0 / are not stored (clim % 8 == 0).  rmod > 0: source row = (r0 + row) % rmod
// (the L noise planes share the data rows).  GI: source column c goes to tile column
// (c & 31) + 64 (c >> 5) -- the W2 slots of the Gaussian decoder's 32-column interleave.
template <int CW, int W, bool GI = false>
DEV void tile_load(char* t, rsrc_t src, int ld, int r0, int c0, int rlim, int clim, int rmod) {
    constexpr int CPR = CW / 8;                // 16-B chunks per row
    constexpr int N = BM * CPR / NTHR;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int id = threadIdx.x + NTHR * i;
        const int row = id / CPR, ch = id % CPR;
        const int gr = r0 + row, gc = c0 + ch * 8;
        const int sr = rmod > 0 ? gr % rmod : gr;
        const uint32_t off = (gr < rlim && gc < clim) ? ((uint32_t)sr * (uint32_t)ld + (uint32_t)gc) * 2u : kOOB;
        const v4u v = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(src, off, 0, 0));
        const int tc = GI ? ((ch * 8) & 31) + ((ch * 8) >> 5) * 64 : ch * 8;
        *reinterpret_cast<v4u*>(t + row * epitch<W>() + tc * 2) = v;
    }
}
template <int W>
DEV void tile_store(const char* t, bf16_t* dst, int ld, int r0, int c0, int rlim, int clim) {
    constexpr int CPR = W / 8;
    constexpr int N = BM * CPR / NTHR;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int id = threadIdx.x + NTHR * i;
        const int row = id / CPR, ch = id % CPR;
        const int gr = r0 + row, gc = c0 + ch * 8;
        if (gr < rlim && gc < clim)
            *reinterpret_cast<v4u*>(dst + (int64_t)gr * ld + gc) =
                *reinterpret_cast<const v4u*>(t + row * epitch<W>() + ch * 16);
    }
}

// ------------------------------------------------------------------ epilogues
// Interface (W = the block's tile width): static constexpr bool kIn, kOut;
// void load_in<W>(m0, n0, smem) (kIn);  void apply<W>(mw, nw, acc, kz, smem);
// void store_out<W>(m0, n0, smem) (kOut).  A wave's 64 x 64 block starts at tile-local
// (mw & (BM - 1), nw & (W - 1)).
// Plain fp32 store (split-K slabs: slice kz at out + kz * slab).
struct EpiF32 {
    static constexpr bool kIn = false, kOut = false;
    float* out; int ldo; int M, N; int64_t slab;
    template <int W, class CM = ColStd>
    DEV void apply(int mw, int nw, f32x4 (&acc)[4][4], int kz, char*) const {
        const int lane = threadIdx.x & 63;
        float* o = out + (int64_t)kz * slab;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = erow(mw, i, r, lane), col = ecol<CM>(nw, j, lane);
                    if (row < M && col < N) o[(int64_t)row * ldo + col] = acc[i][j][r];
                }
    }
};

// v = act(acc + bias[col]) stored as bf16 (via the LDS tile, 16-B stores).
// tanh for a bf16 result: 1 - 2 / (1 + e^{2x}) for |x| >= 2^-6 (absolute error ~1e-7, far
// below the bf16 spacing), x itself below (|tanh x - x| < x^3 / 3: relative 8e-5 at 2^-6,
// 1/100 of a bf16 ulp) -- two transcendentals and five simple ops, against ftanh's eleven
// (ftanh keeps fp32 accuracy near 0 for the fp32 engine).  The encoder's and dechid's tanh
// epilogues cost ~9 and ~7 us of config 5's step (timing-only build without them).
DEV float ftanh_bf(float x) {
    const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * (2.f * kLog2e)));
    return __builtin_fabsf(x) < 0.015625f ? x : t;
}

struct EpiBiasAct {
    static constexpr bool kIn = false, kOut = true;
    const float* bias; int tanh_act; int M, N;
    bf16_t* out; int ldo;
    template <int W, class CM = ColStd>
    DEV void apply(int mw, int nw, f32x4 (&acc)[4][4], int, char* smem) const {
        const int lane = threadIdx.x & 63;
        const int lr0 = mw & (BM - 1), lc0 = nw & (W - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = ecol<CM>(nw, j, lane);
            const float b = col < N ? bias[col] : 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = acc[i][j][r] + b;
                    if (tanh_act) v = ftanh_bf(v);
                    lds_st_bf<W>(smem, erow(lr0, i, r, lane), ecol<CM>(lc0, j, lane), v);
                }
        }
    }
    template <int W>
    DEV void store_out(int m0, int n0, char* smem) const { tile_store<W>(smem, out, ldo, m0, n0, M, N); }
};

// Backward through tanh: out = acc * (1 - t^2) with t the stored bf16 activation at the
// same (row, col), staged through the LDS tile and overwritten there by the result;
// column sums of out (fp32, before rounding) -> colpart[mw/64][col] (the bias gradient,
// reduced in fixed order by the optimizer).
struct EpiDTanh {
    static constexpr bool kIn = true, kOut = true;
    const bf16_t* t; int ldt; int M, N;
    bf16_t* out; int ldo;
    float* colpart;
    template <int W>
    DEV void load_in(int m0, int n0, char* smem) const {
        tile_load<W, W>(smem, mkbuf(t, (int64_t)M * ldt * 2), ldt, m0, n0, M, N, 0);
    }
    template <int W, class CM = ColStd>
    DEV void apply(int mw, int nw, f32x4 (&acc)[4][4], int, char* smem) const {
        const int lane = threadIdx.x & 63;
        const int lr0 = mw & (BM - 1), lc0 = nw & (W - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = ecol<CM>(nw, j, lane);
            float cs = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int lr = erow(lr0, i, r, lane), lc = ecol<CM>(lc0, j, lane);
                    const float tv = lds_bf<W>(smem, lr, lc);
                    const float v = acc[i][j][r] * (1.f - tv * tv);
                    lds_st_bf<W>(smem, lr, lc, v);
                    cs += (erow(mw, i, r, lane) < M) ? v : 0.f;
                }
            cs = colsum_lanes(cs);
            if (lane < 16 && col < N) colpart[(int64_t)(mw >> 6) * N + col] = cs;
        }
    }
    template <int W>
    DEV void store_out(int m0, int n0, char* smem) const { tile_store<W>(smem, out, ldo, m0, n0, M, N); }
};

// EpiDTanh on the TRANSPOSED product out^T (A' = the weight, B' = the data gradient; the
// block tile is 256 output columns x W output rows): a lane's registers r = 0..3 of fragment
// (i, j) are four consecutive output columns mw + 16 i + 4 q + r of output row nw + CM::off(j)
// + (l & 15), so t is read and out written through the LDS tile with one 8-byte access per
// four elements instead of a 2-byte access per element.  Column sums of out (fp32, before
// rounding) per wave block -> colpart[CM::slot(nw)][col] (the 64 output rows of the wave:
// contiguous with ColStd, two 32-row pieces with Col8; CM::slot numbers them 0.. per 256 rows).
struct EpiDTanhT {
    static constexpr bool kIn = true, kOut = true;
    const bf16_t* t; int ldt; int M, N;   // output rows, output columns (N % 8 == 0)
    bf16_t* out; int ldo;
    float* colpart;
    static constexpr int kPitch = 528;    // 256 bf16 + 16 B: 132 dwords = 4 (mod 64)
    template <int W>
    DEV void load_in(int m0, int n0, char* smem) const {
        const rsrc_t src = mkbuf(t, (int64_t)M * ldt * 2);
        constexpr int CPR = BM / 8, NL = W * CPR / NTHR;
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            const int id = threadIdx.x + NTHR * i;
            const int row = id / CPR, ch = id % CPR;
            const int gr = n0 + row, gc = m0 + ch * 8;
            const uint32_t off = (gr < M && gc < N) ? ((uint32_t)gr * (uint32_t)ldt + (uint32_t)gc) * 2u : kOOB;
            *reinterpret_cast<v4u*>(smem + row * kPitch + ch * 16) =
                __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(src, off, 0, 0));
        }
    }
    template <int W, class CM = ColStd>
    DEV void apply(int mw, int nw, f32x4 (&acc)[4][4], int, char* smem) const {
        const int lane = threadIdx.x & 63, q = lane >> 4, li = lane & 15;
        const int lc0 = mw & (BM - 1), lr0 = nw & (W - 1);
        f32x4 cs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) cs[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = nw + CM::off(j) + li;
            const bool rok = row < M;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const bool ok = rok && mw + 16 * i + 4 * q < N;
                char* px = smem + (lr0 + CM::off(j) + li) * kPitch + (lc0 + 16 * i + 4 * q) * 2;
                const uint2 tr = *reinterpret_cast<const uint2*>(px);
                const float tv[4] = {bf2f(tr.x & 0xFFFFu), bf2f(tr.x >> 16), bf2f(tr.y & 0xFFFFu), bf2f(tr.y >> 16)};
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[i][j][r] * (1.f - tv[r] * tv[r]);
                    cs[i][r] += ok ? v[r] : 0.f;
                }
                *reinterpret_cast<uint2*>(px) = make_uint2(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]));
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int col = mw + 16 * i + 4 * q;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = sum16(cs[i][r]);
                if (li == 0 && col < N) colpart[(int64_t)CM::slot(nw) * N + col + r] = v;
            }
        }
    }
    template <int W>
    DEV void store_out(int m0, int n0, char* smem) const {
        constexpr int CPR = BM / 8, NL = W * CPR / NTHR;
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            const int id = threadIdx.x + NTHR * i;
            const int row = id / CPR, ch = id % CPR;
            const int gr = n0 + row, gc = m0 + ch * 8;
            if (gr < M && gc < N)
                *reinterpret_cast<v4u*>(out + (int64_t)gr * ldo + gc) = *reinterpret_cast<const v4u*>(smem + row * kPitch + ch * 16);
        }
    }
};

// EpiDTanhT for dhd with dz fused into the block (VAEB_BF_DZFUSE): after the tanh backward the
// LDS tile holds dA1 for the block's 256 rows x 256 hidden units (bf16, as stored), so the block
// also forms the split-K partial dZ[rows][Z] = dA1[rows][h-tile] W1[:, h-tile]^T over its 256 h:
// wave w takes latents 16 w .. + 15 for all 16 row tiles (A fragments from the LDS tile, B from
// the K-contiguous W1 shadow in L2), 128 MFMAs, and stores the fp32 partial as slab m0 / 256 of
// dz_slab (the layout of the split-K dz GEMM that latent_bwd_v4_kernel sums in slab order).  The
// thin dz launch (its ~0.77 MB of LDS-DMA per CU) is then not needed.
struct EpiDTanhTDz : EpiDTanhT {
    static constexpr bool kPost = true;
    const bf16_t* w1; int Z, H;          // W1 shadow [Z][H]
    float* dz_slab; int64_t slab;        // slab stride (rows x Z floats)
    DEV void post(int m0, int n0, char* smem) const {
        const int lane = threadIdx.x & 63, q = lane >> 4, li = lane & 15;
        const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        if (16 * w >= Z) return;
        const rsrc_t bw = mkbuf(w1, (int64_t)Z * H * 2);
        const int z = 16 * w + li;
        f32x4 acc[16];
#pragma unroll
        for (int rt = 0; rt < 16; ++rt) acc[rt] = zero4();
#pragma unroll 2
        for (int ks = 0; ks < 8; ++ks) {
            const int h = m0 + 32 * ks + 8 * q;
            const bf16x8 bfr = __builtin_bit_cast(
                bf16x8, __builtin_amdgcn_raw_buffer_load_b128(bw, (z < Z && h < H) ? ((uint32_t)z * (uint32_t)H + (uint32_t)h) * 2u : kOOB, 0, 0));
#pragma unroll
            for (int rt = 0; rt < 16; ++rt) {
                const bf16x8 af = *reinterpret_cast<const bf16x8*>(smem + (16 * rt + li) * kPitch + (32 * ks + 8 * q) * 2);
                acc[rt] = mfma16(af, bfr, acc[rt]);
            }
        }
        float* out = dz_slab + (int64_t)(m0 >> 8) * slab;
#pragma unroll
        for (int rt = 0; rt < 16; ++rt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = n0 + 16 * rt + 4 * q + r;
                if (row < M && z < Z) out[(int64_t)row * Z + z] = acc[rt][r];
            }
    }
};

// Decoder output (VAEB.py:257-263, 302-313) on the [M_e x Dn] block of a2 (| a6):
//  Bernoulli: a = acc + b2; log p += x a - softplus(a); dA2 = sl (x - sigmoid(a)).
//  Gaussian : columns interleave in 32-wide groups ([W2 cols | W6 cols] per 64), so a
//             wave's tiles j and j + 2 hold a2 and a6 of the same 32 data columns:
//             y = sigmoid(a2), r = x - y, log p += -1/2 log 2pi - a6/2 - r^2 e^-a6 / 2,
//             dA2 = sl r e^-a6 y (1 - y), dA6 = sl (-1/2 + r^2 e^-a6 / 2).
// The x tile (the block's data columns) is staged in the LDS output tile at the dA2
// positions and overwritten there by dA2 (| dA6) by the lane that read it.  Per-row log p
// partials -> lp[row * nlp + nw/64]; bias-gradient column sums of dA ->
// colpart[mw/64][col]; y (decoder mean, reconstruction) when yout != nullptr.
template <bool GAUSS>
struct EpiDecOut {
    static constexpr bool kIn = true, kOut = true;
    const float *b2, *b6;
    const bf16_t* x; int ldx; int Mx;   // data row of output row m is m % Mx
    int M, N, D;                        // N = Dn (D or 2D)
    int train;
    float sl;                           // sc / L
    BatchRef xb;                        // device-resolved minibatch offset of x
    bf16_t* dA; int ldd;
    float* lp; int nlp;
    float* colpart;
    float* yout;
    template <int W>
    DEV void load_in(int m0, int n0, char* smem) const {
        const rsrc_t src = mkbuf(x + xb.offset(), (int64_t)Mx * ldx * 2);
        if constexpr (GAUSS) tile_load<W / 2, W, true>(smem, src, ldx, m0, n0 / 2, M, D, Mx);
        else tile_load<W, W>(smem, src, ldx, m0, n0, M, D, Mx);
    }
    template <int W, class CM = ColStd>
    DEV void apply(int mw, int nw, f32x4 (&acc)[4][4], int, char* smem) const {
        static_assert(!GAUSS || CM::off(2) == 32, "the Gaussian interleave pairs tiles j and j + 2, 32 columns apart");
        const int lane = threadIdx.x & 63;
        const int lr0 = mw & (BM - 1), lc0 = nw & (W - 1);
        // fragment row i outermost: only its 4 row partials and the JN column partials stay
        // live (the transcendental-heavy body then fits the register budget without spills)
        constexpr int JN = GAUSS ? 2 : 4;
        int col[JN], d[JN];
        bool cok[JN];
        float bb2[JN], bb6[JN], cs2[JN], cs6[JN];
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            col[j] = ecol<CM>(nw, j, lane);                               // dA column
            d[j] = GAUSS ? (nw >> 1) + 16 * j + (lane & 15) : col[j];     // data column
            cok[j] = d[j] < D;
            bb2[j] = cok[j] ? b2[d[j]] : 0.f;
            bb6[j] = (GAUSS && cok[j]) ? b6[d[j]] : 0.f;
            cs2[j] = 0.f;
            cs6[j] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float rs[4] = {0.f, 0.f, 0.f, 0.f};
            float pd[4] = {1.f, 1.f, 1.f, 1.f};   // Bernoulli: prod_j (1 + e^-|a|), one log per row
#pragma unroll
            for (int j = 0; j < JN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = erow(mw, i, r, lane), lr = erow(lr0, i, r, lane);
                    const bool ok = cok[j] && row < M;
                    const float xv = lds_bf<W>(smem, lr, ecol<CM>(lc0, j, lane));
                    const float a2 = acc[i][j][r] + bb2[j];
                    float y, lpv, g2, g6 = 0.f;
                    if constexpr (!GAUSS) {
                        // log p = x a - softplus(a) = x a - max(a, 0) - log(1 + e^-|a|): the
                        // logs of a row's JN elements are taken once, of their product (<= 2^JN)
                        const float t = fexp(-fabsf(a2));
                        const float dd = 1.f + t, rc = frcp(dd);
                        y = a2 >= 0.f ? rc : t * rc;
                        lpv = xv * a2 - fmaxf(a2, 0.f);
                        pd[r] *= ok ? dd : 1.f;
                        g2 = sl * (xv - y);
                    } else {
                        y = sigmoidf(a2);
                        const float a6 = acc[i][j + 2][r] + bb6[j];
                        const float rr = xv - y, e6 = fexp(-a6);
                        lpv = -kHalfLog2Pi - 0.5f * a6 - 0.5f * rr * rr * e6;
                        g2 = sl * rr * e6 * y * (1.f - y);
                        g6 = sl * (-0.5f + 0.5f * rr * rr * e6);
                    }
                    rs[r] += ok ? lpv : 0.f;
                    if (yout && ok) yout[(int64_t)row * D + d[j]] = y;
                    if (train) {
                        lds_st_bf<W>(smem, lr, ecol<CM>(lc0, j, lane), g2);
                        cs2[j] += ok ? g2 : 0.f;
                        if constexpr (GAUSS) {
                            lds_st_bf<W>(smem, lr, ecol<CM>(lc0, j, lane) + 32, g6);
                            cs6[j] += ok ? g6 : 0.f;
                        }
                    }
                }
            if (nw < N) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (!GAUSS) rs[r] -= flog(pd[r]);
                    const float sr = sum16(rs[r]);
                    const int row = erow(mw, i, r, lane);
                    if ((lane & 15) == 0 && row < M) lp[(int64_t)row * nlp + CM::slot(nw)] = sr;
                }
            }
        }
        if (train) {
#pragma unroll
            for (int j = 0; j < JN; ++j) {
                const float c2 = colsum_lanes(cs2[j]);
                if (lane < 16 && cok[j]) colpart[(int64_t)(mw >> 6) * N + col[j]] = c2;
                if constexpr (GAUSS) {
                    const float c6 = colsum_lanes(cs6[j]);
                    if (lane < 16 && cok[j]) colpart[(int64_t)(mw >> 6) * N + col[j] + 32] = c6;
                }
            }
        }
    }
    template <int W>
    DEV void store_out(int m0, int n0, char* smem) const {
        if (train) tile_store<W>(smem, dA, ldd, m0, n0, M, N);
    }
};

// Bernoulli decoder output (VAEB.py:257-263, 302-313) on the TRANSPOSED product
// a2^T = W2^T hd^T (gemm_body with A' = W2 K-outer, B' = hd K-contiguous; a block tile is 256
// output columns x W output rows).  A lane's accumulator registers r = 0..3 of fragment (i, j)
// are then four CONSECUTIVE output columns mw + 16 i + 4 q + r of ONE output row nw + 16 j +
// (l & 15), so the x reads and dA writes through the LDS tile are one 8-byte access per four
// elements (EpiDecOut: a 2-byte access per element -- 15 us of config 5's decoder in a
// timing-only build without them), the bias is one 16-byte load, y one 16-byte store, and a
// row's log p terms stay in the lane (16 elements per wave block, one log of their product).
// Same outputs: lp[row * nlp + col / 64], colpart[row / 64][col], dA (bf16), y.
struct EpiDecOutT {
    static constexpr bool kIn = true, kOut = true;
    const float* b2;
    const bf16_t* x; int ldx; int Mx;   // data row of output row m is m % Mx
    int M, D;                           // output rows, output columns (D % 8 == 0)
    int train;
    float sl;                           // sc / L
    BatchRef xb;
    bf16_t* dA; int ldd;
    float* lp; int nlp;
    float* colpart;
    float* yout;                        // 16-byte aligned or null
    // x as bits [rows][ldx / 32] (the dataset is binary, ldx % 32 == 0; same rows as x, same
    // BatchRef), or null: the tile is then expanded from 8 KiB instead of fetched as 128 KiB --
    // a timing-only build without the x fetch put it at ~11 us of config 5's 142-us decoder
    // (profiles/r6/decoder_xpf_ab.txt)
    const uint32_t* xbits;
    // LDS tile [W rows][256 columns] bf16, pitch 528 B = 132 dwords = 4 (mod 64): the 8-byte
    // accesses of a 32-lane group (16 rows x 2 column quads) hit 64 distinct banks
    static constexpr int kPitch = 528;
    template <int W>
    DEV void load_in(int m0, int n0, char* smem) const {
        if (xbits) {
            // thread t: tile row t / 2, columns 128 (t & 1) .. + 127 = four words; a word past D
            // (a tail tile) or a row past M reads 0, as the 16-bit path's out-of-range chunks
            static_assert(W == 256 && NTHR == 512, "bit tile: 256 rows x 2 halves");
            const int wpr = ldx >> 5;   // words per data row
            const rsrc_t src = mkbuf(xbits + xb.offset() / 32, (int64_t)Mx * wpr * 4);
            const int row = (int)threadIdx.x >> 1, hf = (int)threadIdx.x & 1;
            const int gr = n0 + row, w0 = (m0 >> 5) + 4 * hf;
            const uint32_t one = f2bf(1.f);
            uint32_t wv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                wv[k] = __builtin_amdgcn_raw_buffer_load_b32(
                    src, (gr < M && (w0 + k) * 32 < D) ? ((uint32_t)(gr % Mx) * (uint32_t)wpr + (uint32_t)(w0 + k)) * 4u : kOOB, 0, 0);
            char* dst = smem + row * kPitch + hf * 256;
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) {   // 8 columns (16 bytes) per store
                    const uint32_t b8 = wv[k] >> (8 * q);
                    v4u v;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        v[e] = ((b8 >> (2 * e)) & 1u ? one : 0u) | ((b8 >> (2 * e + 1)) & 1u ? one << 16 : 0u);
                    *reinterpret_cast<v4u*>(dst + (k * 32 + q * 8) * 2) = v;
                }
            return;
        }
        const rsrc_t src = mkbuf(x + xb.offset(), (int64_t)Mx * ldx * 2);
        constexpr int CPR = BM / 8, N = W * CPR / NTHR;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int id = threadIdx.x + NTHR * i;
            const int row = id / CPR, ch = id % CPR;
            const int gr = n0 + row, gc = m0 + ch * 8;
            const uint32_t off = (gr < M && gc < D) ? ((uint32_t)(gr % Mx) * (uint32_t)ldx + (uint32_t)gc) * 2u : kOOB;
            *reinterpret_cast<v4u*>(smem + row * kPitch + ch * 16) =
                __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(src, off, 0, 0));
        }
    }
    template <int W, class CM = ColStd>
    DEV void apply(int mw, int nw, f32x4 (&acc)[4][4], int, char* smem) const {
        const int lane = threadIdx.x & 63, q = lane >> 4, li = lane & 15;
        const int lc0 = mw & (BM - 1), lr0 = nw & (W - 1);
        const rsrc_t bb = mkbuf(b2, (int64_t)D * 4);
        const rsrc_t yb = mkbuf(yout, yout ? (int64_t)M * D * 4 : 0);
        // output row tiles j outermost: the row's log p terms are two running values, the
        // column sums 16 (4 column quads x 4) carried over the row tiles
        f32x4 cs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) cs[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = nw + CM::off(j) + li;
            const bool rok = row < M;
            float rs = 0.f, pd = 1.f;   // pd: prod (1 + e^-|a|) of the row's <= 16 elements (< 2^16)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int col = mw + 16 * i + 4 * q;
                const bool ok = rok && col < D;
                const f32x4 bias = bld4(bb, col < D ? (uint32_t)col * 4u : kOOB);
                char* px = smem + (lr0 + CM::off(j) + li) * kPitch + (lc0 + 16 * i + 4 * q) * 2;
                const uint2 xr = *reinterpret_cast<const uint2*>(px);
                float gv[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t xw = r < 2 ? xr.x : xr.y;
                    const float xv = bf2f((r & 1) ? xw >> 16 : xw & 0xFFFFu);
                    const float a = acc[i][j][r] + bias[r];
                    const float t = fexp(-fabsf(a));
                    const float dd = 1.f + t, rc = frcp(dd);
                    const float y = a >= 0.f ? rc : t * rc;
                    rs += ok ? xv * a - fmaxf(a, 0.f) : 0.f;
                    pd *= ok ? dd : 1.f;
                    const float g = sl * (xv - y);
                    cs[i][r] += ok ? g : 0.f;
                    if (yout && ok) bst(yb, (uint32_t)(row * D + col + r) * 4u, y);
                    gv[r] = g;
                }
                if (train) *reinterpret_cast<uint2*>(px) = make_uint2(f2bf2(gv[0], gv[1]), f2bf2(gv[2], gv[3]));
            }
            float v = rs - flog(pd);
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            if (q == 0 && rok && mw < D) lp[(int64_t)row * nlp + (mw >> 6)] = v;
        }
        if (train) {
            // the column sums of this wave block's 64 rows: 4 row tiles in the lane, then the 16
            // lanes of the column quad
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int col = mw + 16 * i + 4 * q;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = sum16(cs[i][r]);
                    if (li == 0 && col < D) colpart[(int64_t)CM::slot(nw) * D + col + r] = v;
                }
            }
        }
    }
    template <int W>
    DEV void store_out(int m0, int n0, char* smem) const {
        if (!train) return;
        constexpr int CPR = BM / 8, N = W * CPR / NTHR;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int id = threadIdx.x + NTHR * i;
            const int row = id / CPR, ch = id % CPR;
            const int gr = n0 + row, gc = m0 + ch * 8;
            if (gr < M && gc < D)
                *reinterpret_cast<v4u*>(dA + (int64_t)gr * ldd + gc) = *reinterpret_cast<const v4u*>(smem + row * kPitch + ch * 16);
        }
    }
};

// Where element (m, n) of a weight-gradient product lives in the reference-order fp32
// arena.  mode 0: one array [M x N]; mode 1: [W4 | W5] column split at n0 (each
// [H x n0]); mode 2: the Gaussian decoder's 32-column interleave of [W2 | W6].
struct ColMap {
    int mode, n0;
    int64_t off0, off1;
    int ld0, ld1;
    DEV int64_t at(int m, int n) const {
        if (mode == 0) return off0 + (int64_t)m * ld0 + n;
        if (mode == 1) return n < n0 ? off0 + (int64_t)m * ld0 + n : off1 + (int64_t)m * ld1 + (n - n0);
        const int seg = (n >> 5) & 1, d = ((n >> 6) << 5) | (n & 31);
        return (seg ? off1 : off0) + (int64_t)m * (seg ? ld1 : ld0) + d;
    }
};

// Weight update from the data gradient dsg of one element (VAEB.py:386-444):
// g = dsg - prior theta; acc += g^2; theta' = theta + lr g / (sqrt(acc) + eps) - decay theta^2.
// gs: the backward's loss scale undone (the fp16 engine carries the 16-bit data gradients
// scaled by a power of two, 1 / gs, so that the mean objective's 1/B-sized gradients stay
// normal fp16 numbers; exact: a power of two); the stored gradient is the unscaled one.
struct Opt {
    const float* th_in; float* th_out; float* accum; float* grad;
    bf16_t* shadow_out;   // 16-bit copy of theta' in GEMM layout (index m * N + n)
    float lr, eps, prior, decay;
    int update, store_grad;
    int64_t n;            // arena elements (buffer-descriptor extent)
    float gs = 1.f;       // gradient unscale (1: none)
    DEV void apply(int64_t idx, int64_t sidx, float dsg) const {   // sidx < 0: no shadow
        dsg *= gs;
        if (store_grad) grad[idx] = dsg;
        if (!update) return;
        const float th = th_in[idx];
        float a = accum[idx];
        const float gg = dsg - prior * th;
        a += gg * gg;
        const float tn = th + lr * gg / (__builtin_amdgcn_sqrtf(a) + eps) - decay * th * th;
        accum[idx] = a;
        th_out[idx] = tn;
        if (sidx >= 0) shadow_out[sidx] = (bf16_t)f2bf(tn);
    }
};

struct EpiAdagrad {
    static constexpr bool kIn = false, kOut = false;
    ColMap map; Opt opt; int M, N;
    int sld;   // row stride of the bf16 shadow (0: N; a column range of a wider weight: its width)
    // vec (host-checked: the arena runs, widths and strides multiples of 4, N % 4 == 0): on the
    // 256-wide tiles each wave transposes its 64 x 64 gradient block through its own 17 KiB of
    // the (free) LDS, so a lane updates four consecutive columns of a row with 16-byte theta /
    // accumulator loads and stores and one 8-byte shadow store -- a quarter of the memory
    // instructions of the per-element form
    int vec;
    template <int W, class CM>
    DEV void apply_vec(int mw, int nw, f32x4 (&acc)[4][4], char* smem) const {
        constexpr int TP = 68;   // row pitch (floats): 16-byte rows, the 4-row write groups on disjoint banks
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        float* t = reinterpret_cast<float*>(smem) + wave * (64 * TP);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) t[(16 * i + 4 * (lane >> 4) + r) * TP + 16 * j + (lane & 15)] = acc[i][j][r] * opt.gs;
        const rsrc_t bth = mkbuf(opt.th_in, opt.n * 4), bac = mkbuf(opt.accum, opt.n * 4);
        const rsrc_t bto = mkbuf(opt.th_out, opt.n * 4), bgr = mkbuf(opt.grad, opt.n * 4);
        const int sl = sld ? sld : N;
#pragma unroll
        for (int h = 0; h < 4; ++h) {   // 4 groups of 4 float4 per lane: loads first, then the stores
            uint32_t off[4];
            int64_t so[4];
            f32x4 g[4], th[4], ac[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = (4 * h + u) * 64 + lane;        // float4 e of the 64 x 64 block
                const int lr = e >> 4, c4 = (e & 15) * 4;      // local row, first local column
                const int row = mw + lr, col = nw + CM::off(c4 >> 4) + (c4 & 15);
                const bool ok = row < M && col < N;            // N % 4 == 0: all four or none
                off[u] = ok ? (uint32_t)map.at(row, col) * 4u : kOOB;
                so[u] = ok ? (int64_t)row * sl + col : -1;
                g[u] = *reinterpret_cast<const f32x4*>(t + lr * TP + c4);
                th[u] = bld4(bth, opt.update ? off[u] : kOOB);
                ac[u] = bld4(bac, opt.update ? off[u] : kOOB);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (opt.store_grad) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, g[u]), bgr, off[u], 0, 0);
                if (!opt.update) continue;
                f32x4 a, tn;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float gg = g[u][k] - opt.prior * th[u][k];
                    a[k] = ac[u][k] + gg * gg;
                    tn[k] = th[u][k] + opt.lr * gg / (__builtin_amdgcn_sqrtf(a[k]) + opt.eps) - opt.decay * th[u][k] * th[u][k];
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, a), bac, off[u], 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, tn), bto, off[u], 0, 0);
                if (so[u] >= 0)
                    *reinterpret_cast<uint2*>(opt.shadow_out + so[u]) = make_uint2(f2bf2(tn[0], tn[1]), f2bf2(tn[2], tn[3]));
            }
        }
    }
    // The optimizer rule of Opt::apply on the wave's 64 x 64 block, one 16-row fragment
    // row (16 elements per lane) per memory round trip: all theta / accumulator loads of
    // the fragment row are issued before its stores (buffer loads, masked elements read
    // out of range), instead of a load -> store chain per element that hipcc cannot
    // reorder (theta_in / accum may alias the stores, as far as it can tell).
    template <int W, class CM = ColStd>
    DEV void apply(int mw, int nw, f32x4 (&acc)[4][4], int, char* smem) const {
        if constexpr (W == 256) {
            if (vec) {
                apply_vec<W, CM>(mw, nw, acc, smem);
                return;
            }
        }
        const int lane = threadIdx.x & 63;
        const rsrc_t bth = mkbuf(opt.th_in, opt.n * 4), bac = mkbuf(opt.accum, opt.n * 4);
        const rsrc_t bto = mkbuf(opt.th_out, opt.n * 4), bgr = mkbuf(opt.grad, opt.n * 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t off[4][4];
            float th[4][4], ac[4][4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = erow(mw, i, r, lane), col = ecol<CM>(nw, j, lane);
                    off[j][r] = (row < M && col < N) ? (uint32_t)map.at(row, col) * 4u : kOOB;
                    th[j][r] = bld(bth, opt.update ? off[j][r] : kOOB);
                    ac[j][r] = bld(bac, opt.update ? off[j][r] : kOOB);
                }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = erow(mw, i, r, lane), col = ecol<CM>(nw, j, lane);
                    const float dsg = acc[i][j][r] * opt.gs;
                    if (opt.store_grad) bst(bgr, off[j][r], dsg);
                    if (opt.update) {
                        const float gg = dsg - opt.prior * th[j][r];
                        const float a = ac[j][r] + gg * gg;
                        const float tn = th[j][r] + opt.lr * gg / (__builtin_amdgcn_sqrtf(a) + opt.eps) -
                                         opt.decay * th[j][r] * th[j][r];
                        bst(bac, off[j][r], a);
                        bst(bto, off[j][r], tn);
                        if (off[j][r] != kOOB) opt.shadow_out[(int64_t)row * (sld ? sld : N) + col] = (bf16_t)f2bf(tn);
                    }
                }
        }
    }
};

// ------------------------------------------------------------------ 256^2 8-phase main loop
// The guide's 256 x 256, BK = 64 schedule (cdna_hip_programming.md §5 "The 256² 8-phase
// template"), written for this engine's operand layouts and epilogues.
//  * LDS: two K-tile buffers of 64 KiB; a buffer holds A then B, each as four 8-KiB blocks
//    (k-sub s = 0, 1: k 0..31 / 32..63) x (half h = 0, 1: rows / columns 0..127 / 128..255)
//    at (2 s + h) 8 KiB, every block the 128-row BK = 32 image of TileDma / frag (KC rows
//    of 64 B, KO k-rows of 256 B, swizzled as gemm_body's), so the LDS-DMA and fragment code
//    is shared.  A half-tile = one operand's half = 2 blocks = 2 LDS-DMA per thread.
//  * waves: (wr, wc) = (wave >> 2, wave & 3).  Phase p of a K-tile computes the C quadrant
//    (ah, bh) = (0,0), (0,1), (1,1), (1,0) of the 256 x 256 tile: wave (wr, wc) owns rows
//    ah 128 + wr 64 .. + 64 and columns bh 128 + wc 32 .. + 32 of it, 4 x 2 fragment tiles x
//    2 k-steps = 16 MFMAs.  Fragment reads per phase: 8 A + 4 B (phase 0), 4 B (phase 1),
//    8 A (phase 2), none (phase 3 reuses phase 0's B).
//  * staging: one half-tile per phase, K-tile t's phases stage B_hi(t+1), A_hi(t+1),
//    A_lo(t+2), B_lo(t+2).  Each half is restaged >= 2 phases after its last fragment read
//    (WAR rule under the staggered groups) and read >= 5 phases after its DMA was issued;
//    every phase waits vmcnt(8) (4 half-tiles in flight) before its first barrier, which
//    retires the half the NEXT phase reads (RAW: wait in phase p, read in p + 1 or later).
//    K-tiles past the slice stage out-of-range (zero) DMAs, so the count never changes.
//  * waves 4..7 run one barrier behind waves 0..3 (ping-pong: one group reads fragments
//    while the other's MFMAs run on the same SIMD); s_setprio(1) around the MFMA cluster.
//  * epilogue: the functors of gemm_body with the column map Col8 (a wave's fragment
//    tiles j = 0, 1 at columns wc 32 + 16 j, j = 2, 3 at 128 + wc 32 + 16 (j - 2)).
DEV void vm_wait8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }

// Two-slice split-K of one 256 x 256 tile, combined in the launch: a weight gradient with
// only 128 tiles (config 5: dW2 | dW6, dW3; K = 8192) runs as 256 half-depth blocks, the
// whole chip, instead of 128 full-depth ones.  No block ever waits for one that has not
// reached this point: the first slice to arrive (ticket 0 -> 1) publishes its fp32 partial
// and exits; the second (ticket 1 or 5) waits only for that publication (bit 4) and adds
// it.  The sum is the same bits whichever slice comes first (fp32 a + b == b + a).
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility table, row 1): the partial is
// stored sc1 (16 B per lane, each wave's registers as they stand: lane l of wave w holds the
// same accumulator elements in both slices), every wave drains (vmcnt(0)), the workgroup
// barrier, then one agent-scope add; the consumer polls from one lane, barrier, sc1 loads.
// The consumer resets the ticket.  Returns true in the block that runs the epilogue.
constexpr int kSplitFlag = 139264;   // LDS byte offset past the epilogue tile (lds8_bytes)
DEV bool split2_combine(const GemmArgs& g, int tile, f32x4* acc, int wave, int lane, char* lds_flag) {
    int* sflag = reinterpret_cast<int*>(lds_flag);
    gint* tk = (gint*)(g.ticket + tile);
    const rsrc_t pb = mkbuf(g.part + (int64_t)tile * 65536, 65536 * 4);
    const uint32_t base = ((uint32_t)wave * 32 * 64 + (uint32_t)lane) * 16u;   // element q at base + q KiB
    if (threadIdx.x == 0) *sflag = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int old = *sflag;
    if (old == 0) {
#pragma unroll
        for (int q = 0; q < 32; ++q) bst4x<16>(pb, base + q * 1024u, acc[q]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(tk, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
    }
    if (threadIdx.x == 0 && !(old & 4)) {
        // bounded: the producer is past its main loop, storing 256 KiB
        for (int n = 0; n < (1 << 22); ++n) {
            if (__hip_atomic_load(tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 4) break;
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the partial's loads below the poll
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // two rounds of 16 loads in flight (register budget)
        f32x4 p[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) p[q] = bld4x<16>(pb, base + (16 * h + q) * 1024u);
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[16 * h + q] += p[q];
    }
    if (threadIdx.x == 0) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

template <int LA, int LB, class Epi>
DEV void gemm8_body(const GemmArgs& g, const Epi& e, int bid, int kz, char* smem) {
    constexpr int BK8 = 64, kBlock = 8192, kOperand = 4 * kBlock, kBuf = 2 * kOperand;
    int tm, tn;
    tile_of(g, bid, tm, tn);
    const int m0 = tm * BM, n0 = tn * 256;
    const int kbeg = kz * g.kslice;
    const int kend = min(g.K, kbeg + g.kslice);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const v4i da = mkdesc(g.A + g.ab.offset(), g.a_bytes), db = mkdesc(g.B, g.b_bytes);
    const TileDma<LA, 128> la[2] = {{da, g.lda, g.M, kend, m0}, {da, g.lda, g.M, kend, m0 + 128}};
    const TileDma<LB, 128> lb[2] = {{db, g.ldb, g.N, kend, n0}, {db, g.ldb, g.N, kend, n0 + 128}};
    // half-tile h of operand op (0 = A, 1 = B) of K-tile t
    auto stage = [&](int op, int h, int t) {
        char* img = smem + (t & 1) * kBuf + op * kOperand + h * kBlock;
        const int k0 = kbeg + t * BK8;
        if (op == 0) {
            la[h].issue(img, k0, wave, lane);
            la[h].issue(img + 2 * kBlock, k0 + 32, wave, lane);
        } else {
            lb[h].issue(img, k0, wave, lane);
            lb[h].issue(img + 2 * kBlock, k0 + 32, wave, lane);
        }
    };
    f32x4 acc[2][2][4][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[a][b][i][j] = zero4();
    bf16x8 af[4][2], bf0[2][2], bf1[2][2];
    auto read_a = [&](const char* buf, int h) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i][kk] = frag<LA, 128>(buf + (2 * kk + h) * kBlock, wr * 64 + 16 * i, 0, lane);
    };
    auto read_b = [&](const char* buf, int h, bf16x8 (&bf)[2][2]) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                bf[j][kk] = frag<LB, 128>(buf + kOperand + (2 * kk + h) * kBlock, wc * 32 + 16 * j, 0, lane);
    };
    auto mma = [&](f32x4 (&c)[4][2], const bf16x8 (&bf)[2][2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    c[i][j] = mfma16(af[i][kk], bf[j][kk], c[i][j]);
        __builtin_amdgcn_s_setprio(0);
    };
    // first barrier of a phase (after its reads, its stage and the counted wait), the
    // fragment reads retired, the MFMA cluster, the second barrier
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    const int nkt = (kend - kbeg + BK8 - 1) / BK8;
    // prologue: K-tile 0 whole, then A_lo(1), B_lo(1); A_lo(0), B_lo(0) certified
    stage(0, 0, 0);
    stage(1, 0, 0);
    stage(1, 1, 0);
    stage(0, 1, 0);
    stage(0, 0, 1);
    stage(1, 0, 1);
    vm_wait8();
    bar();
    if (wr == 1) bar();
    for (int t = 0; t < nkt; ++t) {
        const char* buf = smem + (t & 1) * kBuf;
        // phase 0: quadrant (0, 0); stage B_hi(t + 1)
        read_a(buf, 0);
        read_b(buf, 0, bf0);
        stage(1, 1, t + 1);
        vm_wait8();
        bar();
        mma(acc[0][0], bf0);
        bar();
        // phase 1: quadrant (0, 1); stage A_hi(t + 1)
        read_b(buf, 1, bf1);
        stage(0, 1, t + 1);
        vm_wait8();
        bar();
        mma(acc[0][1], bf1);
        bar();
        // phase 2: quadrant (1, 1); stage A_lo(t + 2)
        read_a(buf, 1);
        stage(0, 0, t + 2);
        vm_wait8();
        bar();
        mma(acc[1][1], bf1);
        bar();
        // phase 3: quadrant (1, 0) (A_hi and B_lo from registers); stage B_lo(t + 2)
        stage(1, 0, t + 2);
        vm_wait8();
        bar();
        mma(acc[1][0], bf0);
        bar();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the out-of-range tail DMAs
    if (wr == 0) __builtin_amdgcn_s_barrier();          // re-align the groups' barrier counts
    __syncthreads();
    if (g.part) {
        if (!split2_combine(g, bid, &acc[0][0][0][0], wave, lane, smem + kSplitFlag)) return;
        kz = 0;
    }
    if constexpr (Epi::kIn) {
        e.template load_in<256>(m0, n0, smem);
        __syncthreads();
    }
    // the two row halves with compile-time indices (a runtime `ah` put the whole
    // accumulator in scratch for the large epilogues)
    auto half = [&](auto AH) {
        constexpr int ah = decltype(AH)::value;
        f32x4 blk[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) blk[i][j] = acc[ah][j >> 1][i][j & 1];
        e.template apply<256, Col8>(m0 + ah * 128 + wr * 64, n0 + wc * 32, blk, kz, smem);
    };
    half(std::integral_constant<int, 0>{});
    half(std::integral_constant<int, 1>{});
    if constexpr (Epi::kOut) {
        __syncthreads();
        e.template store_out<256>(m0, n0, smem);
    }
    if constexpr (HasPost<Epi>::value) e.post(m0, n0, smem);
}

template <int LA, int LB, class Epi>
__global__ __launch_bounds__(NTHR, 2) void gemm8_kernel(GemmArgs g, Epi e) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    gemm8_body<LA, LB, Epi>(g, e, blockIdx.x, blockIdx.y, smem);
}
// Two products in one grid on the 8-phase loop (gemm2_kernel's dhd ∥ dW2 grid)
template <int LA1, int LB1, class E1, int LA2, int LB2, class E2>
__global__ __launch_bounds__(NTHR, 2) void gemm8x2_kernel(GemmArgs g1, E1 e1, GemmArgs g2, E2 e2, int nb1) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int b = blockIdx.x;
    if (b < nb1) gemm8_body<LA1, LB1, E1>(g1, e1, b, 0, smem);
    else gemm8_body<LA2, LB2, E2>(g2, e2, b - nb1, 0, smem);
}
// dynamic LDS of gemm8_kernel: the two K-tile buffers, or the 256-wide epilogue tile
// (+ 16 B: the split-K ticket value, kSplitFlag)
constexpr int lds8_bytes() { return ((2 * 65536 > BM * epitch<256>()) ? 2 * 65536 : BM * epitch<256>()) + 16; }
static_assert(BM * epitch<256>() == kSplitFlag && 2 * 65536 <= kSplitFlag, "split-K flag slot");

}  // namespace VAEB_H16NS
}  // namespace vaeb
