// Horizontally fused launches: a critical-path phase and an off-path weight-gradient
// group share one grid, so the weight-gradient tiles run on the CUs the narrow phase
// leaves idle, with no extra kernel boundary and no cross-stream dependency (a forked
// side stream inside a hipGraph measured ~12 us/step slower than one stream).
//
//   P5  (dhd, 224 tiles at MNIST-20) + dW2|dW6 (104 tiles)   -- both need only P4's output
//   P67 (dz/dh, 7 row blocks x 8 column splits) + dW1 (8 tiles) -- both need only P5's output
//
// In the dhd | dW2 launch the weight-gradient blocks are dispatched first, in the dz/dh |
// dW1 launch the phase blocks; all blocks are 512 threads, so the weight-gradient tiles
// use the 8-wave K-split form.
#pragma once
#include "fused.hpp"
#include "kernels_aux.hpp"

namespace vaeb {

template <int WM, int WN, int KS, int NB, int GCH, class P, bool VEC, int TS>
__global__ __launch_bounds__(512) void tile_wgrad_kernel(P p0, WGradArgs w, int ntile, int gx) {
    static_assert(WM * WN * KS == 8, "fused launches are 512 threads");
    __shared__ float sa[kWKB][kWP];
    __shared__ float sb[kWKB][kWP];
    // XCD remap within each part: the phase tiles (critical path) stay spread over all
    // XCDs, each XCD's share contiguous in tile order
    // the weight-gradient blocks take the low block indices (dispatched first: their
    // Adagrad epilogue makes them the longer pole; dhd | dW2 8.55 vs 9.12 us)
    const int nwg = w.total_wgs - ntile;   // grid = w.total_wgs
    const int b0 = (int)blockIdx.x < nwg ? (int)blockIdx.x + ntile : (int)blockIdx.x - nwg;
    const int bid = b0 < ntile ? xcd_remap(b0, ntile) : ntile + xcd_remap(b0 - ntile, nwg);
    if (bid < ntile) {
        P p = p0;
        VAEB_STAMP(p.a, 0);
        tile_body<WM, WN, KS, NB, GCH, P>(p, bid % gx, bid / gx);
        return;
    }
    if (VAEB_DBG_ON(w.dbg) && threadIdx.x == 0) w.dbg[bid * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    wgrad_body<VEC, 8, TS>(w, w.g[0], bid, sa, sb);
}

template <int NCT, bool VEC, int TS>
__global__ __launch_bounds__(512) void dz_dh_wgrad_kernel(StepArgs a, WGradArgs w, int nrow) {
    __shared__ float sa[kWKB][kWP];
    __shared__ float sb[kWKB][kWP];
    // phase blocks first here (dispatching the dW1 blocks first: MNIST no change, Frey
    // 8.0 -> 8.8 us)
    const int b0 = blockIdx.x;
    const int bid = b0 < nrow ? b0 : nrow + xcd_remap(b0 - nrow, (int)gridDim.x - nrow);
    if (bid < nrow) {   // nrow = row blocks x column splits, split-major
        VAEB_STAMP(a, 0);
        const int nrb = a.Mbp >> 4;
        dz_dh_body<NCT>(a, (bid % nrb) * 16, bid / nrb, nrow / nrb);
        return;
    }
    if (VAEB_DBG_ON(w.dbg) && threadIdx.x == 0) w.dbg[bid * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    wgrad_body<VEC, 8, TS>(w, w.g[0], bid, sa, sb);
}

}  // namespace vaeb
