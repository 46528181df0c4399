/*
 * vaeb_diag.h -- diagnostics and measurement hooks of libvaeb_hip.so.
 *
 * NOT part of the drop-in boundary (include/vaeb_hip.h): these entry points have no
 * counterpart in the reference (/root/reference/VAEB.py).  bench.py uses
 * vaeb_profile_steps / vaeb_kernel_name for the per-kernel times it reports; the rest
 * serves the kernel tests and the A/B scripts under scripts/.
 */
#ifndef VAEB_DIAG_H
#define VAEB_DIAG_H

#include "vaeb_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Measurement: runs n_steps eager steps with HIP events around every launch on the
 * context's stream; writes the average device time (ms) and the kernel id of each
 * launch slot of one step.  vaeb_kernel_name maps a kernel id to its name. */
int vaeb_profile_steps(vaeb_ctx* ctx, int32_t n_steps, float* out_ms_per_kernel,
                       int32_t* out_kernel_ids, int32_t max_kernels, int32_t* out_n_kernels);
int vaeb_kernel_name(int32_t kernel_id, char* out, int32_t cap);

/* How the context's steps run: graphs disabled by the config, not captured yet (the first
 * vaeb_update / vaeb_update_many captures them), replaying captured graphs, or eager launches
 * after a failed capture (msg: the failure; with a communicator of > 1 ranks a failed capture
 * is an error of the call instead, never a silent fallback). */
enum vaeb_graph_mode { VAEB_GRAPH_OFF = 0, VAEB_GRAPH_NOT_CAPTURED = 1, VAEB_GRAPH_REPLAY = 2,
                       VAEB_GRAPH_EAGER_FALLBACK = 3 };
int vaeb_graph_status(vaeb_ctx* ctx, int32_t* mode, char* msg, int32_t cap);
/* Diagnostics: vaeb_update_many bracketed by events on the context's stream (after a stream
 * sync): the GPU time from the call's first enqueued work to its last, and the host time
 * the call itself took to enqueue (graph launches, the order upload). */
int vaeb_time_update_many(vaeb_ctx* ctx, const int32_t* batch_indices, int32_t n, float* out_gpu_ms,
                          double* out_enqueue_ms);
/* Diagnostics: every CU busy (MFMA loop) for `us` microseconds on the context's stream. */
int vaeb_busy(vaeb_ctx* ctx, int32_t us);
/* Data-parallel configuration: the RCCL version (ncclGetVersion), whether bucket A's
 * all-reduce + Adagrad overlap the backward on a second stream (-1: no communicator), and
 * the communicator's world size (1 without one). */
int vaeb_comm_info(vaeb_ctx* ctx, int32_t* rccl_version, int32_t* dp_overlap, int32_t* world);
/* Host-only diagnostics (no device call, no context): the sharded data-parallel optimizer's
 * index plan exactly as a rank's step computes it (vaeb_hip.hip dp_bucket_*_runs,
 * dp_shard_len, dp_opt_range, dp_foreign_range; the reference's simultaneous Adagrad,
 * VAEB.py:426-444, split over ranks).  bucket: 0 = A (W2 | W6), 1 = B (the rest and the SGVB
 * slot), 2 = all.  sharded: 1 = reduce-scatter / own shard / all-gather, 0 = replicated.
 * Outputs (each may be NULL): out_P the arena length; runs[3 * 3] per run (lo, n, shard
 * length S), out_nrun runs; own[2 * 6] the (lo, n) index runs this rank's optimizer launch
 * updates, out_nown of them, out_book whether it also books the SGVB slot; foreign[2 * 6]
 * the runs other ranks own (the bf16 shadow fix), out_nforeign of them. */
int vaeb_dp_plan(const vaeb_config* cfg, int32_t world, int32_t rank, int32_t sharded, int32_t bucket,
                 int64_t* out_P, int64_t* runs, int32_t* out_nrun, int64_t* own, int32_t* out_nown,
                 int32_t* out_book, int64_t* foreign, int32_t* out_nforeign);
/* Diagnostics: the world > 1 device path of the sharded data-parallel optimizer on ONE GPU.
 * Runs rank `rank` of a `world`-rank step's optimizer for one gradient bucket (0 = A, 1 = B,
 * 2 = all; as vaeb_dp_plan) on a context WITHOUT a communicator, with the collectives of
 * dp_reduce_update replaced by host copies and its kernels and index ranges unchanged:
 *   1. bucket 0 or 2 (a step's first bucket): the out arena (theta' and the bf16 shadow) is
 *      filled with NaN, so every element the step leaves was written by it;
 *   2. the reduce-scatter: grad_sum (P + 1 floats, the summed data gradient | SGVB) is uploaded
 *      to this rank's destinations only (its own shards and the replicated remainders); every
 *      other gradient element is NaN;
 *   3. this rank's optimizer launch over its range (the step's adagrad kernel; bf16: with the
 *      shadow of what it updates); the SGVB bookkeeping is not run;
 *   4. theta_gathered (P floats, may be NULL): the all-gather -- the other ranks' theta' shards
 *      are copied into the out arena -- then (bf16) the shadow rewrite of those elements
 *      (shadow_runs_kernel).
 * finish = 1 flips the arenas as a step does (vaeb_get_params then reads theta').  The
 * Adagrad state is updated in place for this rank's range only (vaeb_get_adagrad_state). */
int vaeb_dp_rank_update(vaeb_ctx* ctx, int32_t world, int32_t rank, int32_t bucket, const float* grad_sum,
                        int64_t n_grad, const float* theta_gathered, int32_t finish);
/* Diagnostics (bf16 engine): the current bf16 shadow of the weight elements, in arena
 * (reference) order; n = the number of weight elements (the arena before the biases). */
int vaeb_get_shadow(vaeb_ctx* ctx, uint16_t* out, int64_t n);
/* Diagnostics: one eager step with a 100 MHz s_memrealtime stamp per workgroup at the
 * stage boundaries of every launch; out = [launch][1024 workgroups][8 slots]. */
int vaeb_debug_timeline(vaeb_ctx* ctx, int32_t batch_index, uint64_t* out, int64_t cap,
                        int32_t* out_launches);

/* Test hook for the bf16 GEMM engine: C[M x N] = sum_k A(m, k) B(k, n) with the operands
 * rounded to bf16 on device.  a_kouter = 0: A is stored [M x K], 1: [K x M]; b_kouter = 0:
 * B is stored [N x K], 1: [K x N].  ksplit K slices are summed in fixed order; ksplit < 0: the
 * 256 x 256 8-phase main loop with -ksplit slices; -22: two slices combined inside the launch
 * (split2_combine).  Uses the context's device and stream. */
int vaeb_test_gemm_bf16(vaeb_ctx* ctx, int32_t a_kouter, int32_t b_kouter, int32_t M, int32_t N, int32_t K,
                        const float* A, const float* B, float* C, int32_t ksplit);
/* Diagnostics: mean time (ms) of `reps` back-to-back launches of the bf16 GEMM on
 * device-generated uniform [-1, 1) operands of the given layouts, bias + bf16-store
 * epilogue; tile width 128 / 256 (0: the engine's choice; 8: 256 x 256 on the 8-phase loop;
 * 9: the same as two K slices combined in the launch). */
int vaeb_bench_gemm_bf16(vaeb_ctx* ctx, int32_t a_kouter, int32_t b_kouter, int32_t M, int32_t N, int32_t K,
                         int32_t tile_n, int32_t reps, float* out_ms);

#ifdef __cplusplus
}
#endif
#endif /* VAEB_DIAG_H */
