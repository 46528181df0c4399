// h16_engines.hpp -- the 16-bit MFMA engine's device code, instantiated for both operand types:
//   namespace vaeb::bf  bf16 operands (v_mfma_f32_16x16x32_bf16)   VAEB_DTYPE_BF16
//   namespace vaeb::hf  fp16 operands (v_mfma_f32_16x16x32_f16)    VAEB_DTYPE_F16 (BASELINE config 5
//                       names "fp16 MFMA"; the same dense rate on gfx950)
// gemm_bf16.hpp, step_bf16.hpp and thin_bf16.hpp are written once against the names bf16_t /
// bf16x8 / f2bf / bf2f / mfma16 and included here twice; the element-type-independent part
// (BfState, ShadowMap, BatchRef) lives in h16_common.hpp.
#pragma once
#include <type_traits>
#include "tile_engine.hpp"
#include "kernels_aux.hpp"
#include "h16_common.hpp"

#define VAEB_H16NS bf
#define VAEB_H16_F16 0
#include "gemm_bf16.hpp"
#include "step_bf16.hpp"
#include "thin_bf16.hpp"
#undef VAEB_H16NS
#undef VAEB_H16_F16

#define VAEB_H16NS hf
#define VAEB_H16_F16 1
#include "gemm_bf16.hpp"
#include "step_bf16.hpp"
#include "thin_bf16.hpp"
#undef VAEB_H16NS
#undef VAEB_H16_F16
