// Diagnostics (not product code): a 256 x 256 GEMM main loop on FOUR waves (one per SIMD,
// 128 x 128 outputs each, 256 accumulator registers) against the engine's 8-wave 8-phase
// ping-pong loop (gemm8_kernel), same operand images (TileDma / frag), same tile order,
// fp16 operands, uniform [-1, 1) data, in one process.
//   4-wave loop: a 4-stage LDS ring of BK = 32 stages (A 16 KiB + B 16 KiB), one barrier per
//   stage; after the barrier that certifies stage t + 1 a wave issues the LDS-DMA of stage
//   t + 3, reads stage t + 1's fragments into the second register set and runs stage t's 64
//   MFMAs from the first (fragments double-buffered in registers across the barrier).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/gemm4w_probe scripts/gemm4w_probe.hip
// Run:   scripts/gemm4w_probe   (prints TF/s per shape and the max error against a float64 sample)
#define VAEB_H16NS hf
#define VAEB_H16_F16 1
#include "../vaeb_amd/csrc/phases.hpp"
#include "../vaeb_amd/csrc/gemm_bf16.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace vaeb {
namespace hf {

DEV void bar_raw() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

template <int LA, int LB>
__global__ __launch_bounds__(256, 1) void g4_kernel(GemmArgs g, float* out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int kA = 256 * 32 * 2, kSt = 2 * kA;
    int tm, tn;
    tile_of(g, blockIdx.x, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const v4i da = mkdesc(g.A, g.a_bytes), db = mkdesc(g.B, g.b_bytes);
    const TileDma<LA, 256> la{da, g.lda, g.M, g.K, m0};
    const TileDma<LB, 256> lb{db, g.ldb, g.N, g.K, n0};
    auto issue = [&](int t) {
        char* st = smem + (t & 3) * kSt;
        const int k0 = t * 32;
        la.issue(st, k0, 2 * wave, lane);
        la.issue(st, k0, 2 * wave + 1, lane);
        lb.issue(st + kA, k0, 2 * wave, lane);
        lb.issue(st + kA, k0, 2 * wave + 1, lane);
    };
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = zero4();
    // registers: B fragments of the stage being multiplied (fb) and of the next (fn); A
    // fragments streamed two rows ahead (fa)
    bf16x8 fb[8], fn[8], fa[8];
    auto st_of = [&](int t) { return smem + (t & 3) * kSt; };
    auto rdA = [&](int t, int i) { fa[i] = frag<LA, 256>(st_of(t), wr * 128 + 16 * i, 0, lane); };
    auto rdB = [&](int t, bf16x8 (&b)[8]) {
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = frag<LB, 256>(st_of(t) + kA, wc * 128 + 16 * j, 0, lane);
    };
    auto rows = [&](int i, const bf16x8 (&b)[8]) {
#pragma unroll
        for (int ii = i; ii < i + 2; ++ii)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[ii][j] = mfma16(fa[ii], b[j], acc[ii][j]);
    };
    const int nkt = g.K / 32;   // the probe's K is a multiple of 64
    issue(0);
    issue(1);
    issue(2);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    bar_raw();
    rdB(0, fb);
    rdA(0, 0);
    rdA(0, 1);
    // stage t: rows 0-5 while A rows 2-7 stream in; certify stage t + 1 (vmcnt + barrier),
    // issue stage t + 3; rows 6-7 while stage t + 1's B fragments and A rows 0-1 stream in
    auto stage = [&](int t, bf16x8 (&b)[8], bf16x8 (&bn)[8]) {
        __builtin_amdgcn_s_setprio(1);
        rdA(t, 2); rdA(t, 3);
        rows(0, b);
        __builtin_amdgcn_sched_barrier(0);
        rdA(t, 4); rdA(t, 5);
        rows(2, b);
        __builtin_amdgcn_sched_barrier(0);
        rdA(t, 6); rdA(t, 7);
        rows(4, b);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // own pieces of stage t + 1
        bar_raw();
        issue(t + 3);
        __builtin_amdgcn_s_setprio(1);
        rdB(t + 1, bn);
        rows(6, b);
        __builtin_amdgcn_sched_barrier(0);
        rdA(t + 1, 0); rdA(t + 1, 1);
        __builtin_amdgcn_s_setprio(0);
    };
    for (int t = 0; t < nkt; t += 2) {
        stage(t, fb, fn);
        stage(t + 1, fn, fb);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wr * 128 + 16 * i + 4 * (lane >> 4) + r, col = n0 + wc * 128 + 16 * j + (lane & 15);
                out[(int64_t)row * g.N + col] = acc[i][j][r];
            }
}

__global__ void fill_kernel(bf16_t* p, int64_t n, uint32_t seed) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t h = (uint32_t)i * 0x9E3779B1u ^ seed;
        h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
        p[i] = (bf16_t)f2bf((float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f);
    }
}

}  // namespace hf
}  // namespace vaeb

using namespace vaeb::hf;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static float h2f(uint16_t h) {
    const uint32_t s = (h >> 15) & 1, e = (h >> 10) & 31, m = h & 1023;
    float v = e == 0 ? std::ldexp((float)m, -24) : std::ldexp((float)(m | 1024), (int)e - 25);
    return s ? -v : v;
}

template <int LA, int LB>
void run_shape(const char* name, int M, int N, int K) {
    bf16_t *A, *B;
    float* C;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 4));
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, A, (int64_t)M * K, 1u);
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, B, (int64_t)N * K, 2u);
    GemmArgs g{};
    g.A = A; g.lda = LA == KO ? M : K; g.a_bytes = (int64_t)M * K * 2;
    g.B = B; g.ldb = LB == KO ? N : K; g.b_bytes = (int64_t)N * K * 2;
    g.M = M; g.N = N; g.K = K;
    g.tiles_m = M / 256; g.tiles_n = N / 256;
    g.kslice = K;
    const int nt = g.tiles_m * g.tiles_n;
    EpiF32 e{C, N, M, N, 0};
    CK(hipFuncSetAttribute((const void*)g4_kernel<LA, LB>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    CK(hipFuncSetAttribute((const void*)gemm8_kernel<LA, LB, EpiF32>, hipFuncAttributeMaxDynamicSharedMemorySize, lds8_bytes()));
    auto l4 = [&]() { hipLaunchKernelGGL((g4_kernel<LA, LB>), dim3(nt), dim3(256), 131072, 0, g, C); };
    auto l8 = [&]() { hipLaunchKernelGGL((gemm8_kernel<LA, LB, EpiF32>), dim3(nt), dim3(512), lds8_bytes(), 0, g, e); };
    // correctness of the 4-wave loop on a sample against float64
    l4();
    CK(hipDeviceSynchronize());
    std::vector<uint16_t> ha((size_t)M * K), hb((size_t)N * K);
    CK(hipMemcpy(ha.data(), A, ha.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), B, hb.size() * 2, hipMemcpyDeviceToHost));
    std::vector<float> hc((size_t)M * N);
    CK(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
    double maxerr = 0;
    for (int s = 0; s < 512; ++s) {
        const int m = (int)((s * 2654435761u) % M), n = (int)((s * 40503u + 7) % N);
        double ref = 0;
        for (int k = 0; k < K; ++k) {
            const float a = h2f(LA == KO ? ha[(size_t)k * M + m] : ha[(size_t)m * K + k]);
            const float b = h2f(LB == KO ? hb[(size_t)k * N + n] : hb[(size_t)n * K + k]);
            ref += (double)a * b;
        }
        maxerr = std::fmax(maxerr, std::fabs(ref - hc[(size_t)m * N + n]));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double fl = 2.0 * M * N * K;
    float t4[3], t8[3];
    for (int r = 0; r < 3; ++r) {
        for (int v = 0; v < 2; ++v) {
            auto go = [&]() { if (v) l8(); else l4(); };
            go();
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 10; ++i) go();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            (v ? t8 : t4)[r] = ms / 10;
        }
    }
    auto med = [](float* t) { float a = t[0], b = t[1], c = t[2]; return std::fmax(std::fmin(a, b), std::fmin(std::fmax(a, b), c)); };
    printf("%-6s M=%d N=%d K=%d: 4-wave %6.0f TF/s  8-phase %6.0f TF/s  (4-wave max |err| %.3g)\n", name, M, N, K,
           fl / (med(t4) * 1e-3) / 1e12, fl / (med(t8) * 1e-3) / 1e12, maxerr);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
}

int main() {
    run_shape<KC, KO>("enc", 8192, 2048, 4096);
    run_shape<KC, KC>("dhd", 8192, 2048, 4096);
    run_shape<KC, KO>("dec", 8192, 4096, 2048);
    run_shape<KO, KO>("dW3", 4096, 2048, 8192);
    return 0;
}
