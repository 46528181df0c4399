// h16_common.hpp -- the element-type-independent part of the 16-bit (bf16 / fp16) engine:
// what the host keeps per context and what the kernels of both instantiations (h16_engines.hpp)
// share.  16-bit values are raw bits in memory (uint16_t) in either format.
#pragma once
#include "tile_engine.hpp"

namespace vaeb {
namespace h16c {

typedef uint16_t h16_t;   // raw 16-bit operand bits (bf16 or fp16, per the context's dtype)

// Device-side minibatch resolution: rows of batch order[*cursor] start `stride`
// elements after the base (the cursor advances in the step's last kernel), so a whole
// epoch replays as graphs with no host round trip.  order == nullptr: offset 0.
struct BatchRef {
    const int* order; const int* cursor; int64_t stride;
    DEV int64_t offset() const { return order ? (int64_t)order[*cursor] * stride : 0; }
};

// Arena (reference order) -> shadow index map.
struct ShadowMap {
    int64_t offW3, offW4, offW5, offW1, offW2, offW6;   // arena offsets (offW6 < 0: Bernoulli)
    int64_t s3, s45, s1, s26;                           // shadow offsets
    int D, H, Z;
    int64_t nweights;                                   // arena elements before the biases
    DEV int64_t at(int64_t i) const {
        if (i >= nweights) return -1;
        const int Z2 = 2 * Z;
        if (i < offW4) return s3 + (i - offW3);
        if (i < offW5) { const int64_t e = i - offW4; return s45 + (e / Z) * Z2 + e % Z; }
        if (i < offW1) { const int64_t e = i - offW5; return s45 + (e / Z) * Z2 + Z + e % Z; }
        if (i < offW2) return s1 + (i - offW1);
        const bool w6 = offW6 >= 0 && i >= offW6;
        const int64_t e = i - (w6 ? offW6 : offW2);
        const int64_t h = e / D, d = e % D;
        if (offW6 < 0) return s26 + h * D + d;
        return s26 + h * 2 * D + ((d >> 5) << 6) + (w6 ? 32 : 0) + (d & 31);
    }
};

// Device buffers of the 16-bit engine (one context).  Row capacity R = max(B, eval chunk).
struct BfState {
    bool on = false;
    int Dn = 0;                        // decoder output width (D, or 2D interleaved)
    int64_t S = 0;                     // shadow elements
    int64_t s3 = 0, s45 = 0, s1 = 0, s26 = 0;
    h16_t* shadow2[2] = {nullptr, nullptr};
    h16_t* x = nullptr;               // dataset [N x D], 16-bit
    h16_t* xeval = nullptr;           // eval chunk [R x D]
    h16_t* xval = nullptr;            // resident validation set [nval x D] (vaeb_set_valid_data)
    // the dataset as bits [N x D / 32] when every value is exactly 0 or 1 and D % 32 == 0 (the
    // Bernoulli decoder epilogue's x tile then costs 1/16 of the bytes; x itself is unchanged)
    uint32_t* xbits = nullptr;
    h16_t *h = nullptr, *z = nullptr, *hd = nullptr, *dA = nullptr, *dA1 = nullptr, *dml = nullptr,
           *dA3 = nullptr;
    float *ml_slab = nullptr, *dz_slab = nullptr, *w_slab = nullptr;
    float *cp3 = nullptr, *cp45 = nullptr, *cp1 = nullptr, *cp26 = nullptr, *lp = nullptr, *kl = nullptr;
    float *mu = nullptr, *lv = nullptr, *eps = nullptr;
    double* elbo_parts = nullptr;      // [kElboBlocks][2] stage-1 ELBO sums
    int ks_heads = 1, ks_dz = 1, ks_w1 = 1, ks_w45 = 1;
    // latent-width products with the latent block fused into their epilogues (thin_bf16.hpp;
    // LB, L = 1, Z % 128 == 0): no split-K slabs; nkl KL partials per row (Z / 64)
    bool thin_h = false, thin_z = false;   // heads / dz on the thin launches
    int nkl = 1;
    ShadowMap smap{};
};

}  // namespace h16c
}  // namespace vaeb
