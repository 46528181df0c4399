// Diagnostics: does a dispatch start with a cold instruction cache?  Same work (a
// dependent chain of N FMAs per lane) as straight-line code (N unrolled: ~8 B per FMA of
// code) and as a loop (a few hundred bytes of code), 224 workgroups x 512 threads (the
// MNIST encoder's grid), each launched back to back; reports mean us per launch.
// Build: hipcc --offload-arch=gfx950 -O3 -o icache_probe icache_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
__global__ __launch_bounds__(512) void straight(float* out, float a, float b) {
    float v = threadIdx.x * 1e-3f;
#pragma unroll
    for (int i = 0; i < N; ++i) v = __builtin_fmaf(v, a + (float)(i & 7) * 1e-7f, b);
    if (v == 12345.f) out[threadIdx.x] = v;
}

__global__ __launch_bounds__(512) void looped(float* out, float a, float b, int n) {
    float v = threadIdx.x * 1e-3f;
    for (int i = 0; i < n; ++i) v = __builtin_fmaf(v, a + (float)(i & 7) * 1e-7f, b);
    if (v == 12345.f) out[threadIdx.x] = v;
}

template <class F>
float time_us(F launch, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 20; ++i) launch();
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return 1000.f * ms / reps;
}

template <int N>
void run(float* d) {
    const float s = time_us([&] { hipLaunchKernelGGL(straight<N>, dim3(224), dim3(512), 0, 0, d, 0.999f, 1e-3f); }, 200);
    const float l = time_us([&] { hipLaunchKernelGGL(looped, dim3(224), dim3(512), 0, 0, d, 0.999f, 1e-3f, N); }, 200);
    // alternate the two kernels: each launch follows a different kernel
    const float alt = time_us([&] {
        hipLaunchKernelGGL(straight<N>, dim3(224), dim3(512), 0, 0, d, 0.999f, 1e-3f);
        hipLaunchKernelGGL(looped, dim3(224), dim3(512), 0, 0, d, 0.999f, 1e-3f, 16);
    }, 200);
    const float l16 = time_us([&] { hipLaunchKernelGGL(looped, dim3(224), dim3(512), 0, 0, d, 0.999f, 1e-3f, 16); }, 200);
    printf("N=%5d straight %7.2f us  loop %7.2f us  straight+tiny alternating %7.2f us (tiny alone %6.2f)\n", N, s, l,
           alt, l16);
}

// per-kernel cost of a graph-replayed chain of 100 tiny launches at a given grid / block
void graph_chain(float* d, int grid, int block) {
    hipStream_t s;
    hipStreamCreate(&s);
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(looped, dim3(grid), dim3(block), 0, s, d, 0.999f, 1e-3f, 16);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int i = 0; i < 3; ++i) hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, s);
    for (int i = 0; i < 10; ++i) hipGraphLaunch(ge, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("graph of 100 tiny kernels, grid %4d x %4d: %6.2f us per kernel\n", grid, block, 1000.f * ms / 1000);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    hipStreamDestroy(s);
}

int main() {
    float* d;
    hipMalloc(&d, 4096);
    graph_chain(d, 1, 64);
    graph_chain(d, 224, 512);
    graph_chain(d, 448, 512);
    graph_chain(d, 473, 256);
    run<16>(d);
    run<256>(d);
    run<1024>(d);
    run<2048>(d);
    run<4096>(d);
    hipFree(d);
    return 0;
}
