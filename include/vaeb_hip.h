/*
 * vaeb_hip.h -- C ABI of the MI355X-native VAEB SGVB training step (libvaeb_hip.so).
 *
 * The reference's operator boundary is the pair of Theano compiled functions built in
 * VAEB.getGradient (/root/reference/VAEB.py:408-422): `update(index) -> SGVB/B`
 * (mutating theta, the Adagrad accumulators and the RNG stream in place) and
 * `validate(x) -> SGVB` (forward-only sum).  This header exports those two operations
 * plus the state transfers the Python `VAEB` class needs (VAEB.py:132-242), as plain
 * `extern "C"` functions over host pointers and sizes.  No torch types appear here.
 *
 * Conventions
 *  - Every function returns int: 0 = ok, < 0 = error; vaeb_last_error() returns a
 *    thread-local message for the last failing call on this thread.
 *  - The caller owns host buffers (copied in/out during the call); the library owns all
 *    device memory.  One context per GPU/rank; calls on one context must be serialised.
 *  - Parameters are flat float32 in the reference order
 *    [W3,W4,W5,W1,W2,(W6),b3,b4,b5,b1,b2,(b6)] (VAEB.py:111-115), each row-major (C order).
 */
#ifndef VAEB_HIP_H
#define VAEB_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum vaeb_decoder   { VAEB_DEC_BERNOULLI = 0, VAEB_DEC_GAUSSIAN = 1 };   /* --continuous, VAEB.py:256 */
enum vaeb_estimator { VAEB_EST_LB = 0, VAEB_EST_LA = 1, VAEB_EST_FV = 2,  /* VAEB.py:378-383 */
                      VAEB_EST_FVS = 3 };  /* extension (not in the reference code): full-variational
                                              with the weight-posterior reparameterisation that
                                              VAEB.sample_variational_params (VAEB.py:127-129)
                                              defines but never calls: theta~ = mu + |sigma| zeta */
enum vaeb_objective { VAEB_OBJ_SUM_PRIOR = 0,                             /* VAEB.py:386-390 */
                      VAEB_OBJ_MEAN_MAP = 1 };                            /* VAEBfullbayes.py:142,183 */
enum vaeb_eps_mode  { VAEB_EPS_PHILOX = 0, VAEB_EPS_HOST = 1 };
enum vaeb_dtype     { VAEB_DTYPE_F32 = 0,      /* fp32 MFMA, the reference's floatX (run_on_gpu.sh:2) */
                      VAEB_DTYPE_BF16 = 1,     /* bf16 MFMA operands, fp32 accumulation and fp32
                                                  master weights / Adagrad state (BASELINE config 5) */
                      VAEB_DTYPE_F16 = 2 };    /* fp16 MFMA operands ("fp16 MFMA", BASELINE config 5),
                                                  the same engine and fp32 state; the mean objective's
                                                  backward carries its 16-bit data gradients scaled by
                                                  a power of two ~ B_global (undone in fp32) */
enum vaeb_status    { VAEB_OK = 0, VAEB_ERR_ARG = -1, VAEB_ERR_HIP = -2, VAEB_ERR_STATE = -3,
                      VAEB_ERR_COMM = -4, VAEB_ERR_NOMEM = -5,
                      VAEB_ERR_NUMERIC = -6 };  /* a step's values left the fixed-point latent hand-off's
                                                   range (NaN / inf / |partial| >= 2^17): those latent
                                                   values were set to NaN; reported by the next
                                                   vaeb_update / vaeb_epoch_elbo, then cleared */

typedef struct vaeb_config {
    int32_t D;            /* input size (784 MNIST, 560 Frey)                         */
    int32_t H;            /* hidden units (--hidden_unit, VAEB.py:542-552)             */
    int32_t Z;            /* latent size (--n_latent)                                  */
    int32_t B;            /* rows this rank processes per step                          */
    int32_t B_global;     /* rows of one global minibatch (= B * world for weak scaling) */
    int32_t row_offset;   /* first row of this rank inside the global minibatch          */
    int32_t L;            /* samples per datapoint (--L)                                 */
    int32_t decoder;      /* enum vaeb_decoder                                           */
    int32_t estimator;    /* enum vaeb_estimator                                         */
    int32_t objective;    /* enum vaeb_objective                                         */
    float   lr;           /* --learning_rate (VAEB.py:31)                                */
    float   adagrad_eps;  /* 1e-6 (VAEB.py:144)                                          */
    int32_t device;       /* HIP device ordinal                                          */
    int32_t max_eval_rows;/* largest x passed to vaeb_validate in one device chunk       */
    int32_t use_graph;    /* 1: replay the step as a captured hipGraph                   */
    int32_t keep_grads;   /* 1: also store each step's data gradient (vaeb_get_grads)    */
    int32_t dtype;        /* enum vaeb_dtype; BF16 needs D, H, Z % 8 == 0 (Gaussian: D % 32)  */
    int32_t reserved[5];
} vaeb_config;

typedef struct vaeb_ctx vaeb_ctx;

const char* vaeb_last_error(void);
int vaeb_version(int32_t* major, int32_t* minor);

/* Lifetime */
int vaeb_create(const vaeb_config* cfg, vaeb_ctx** out);
int vaeb_destroy(vaeb_ctx* ctx);
int vaeb_num_params(const vaeb_ctx* ctx, int64_t* n);

/* Training data: copied into a device-resident store owned by ctx (replaces the
 * th.shared x_train of VAEB.py:184).  Row-major float32 [n_rows x D].  16-bit contexts
 * keep it as fp16 / bf16 and, when every value is exactly 0 or 1 and D % 32 == 0, also as
 * bits (1/16 of that), from which the Bernoulli decoder expands its x tiles: the same
 * values, so the same steps bit for bit (one host pass over x decides). */
int vaeb_set_data(vaeb_ctx* ctx, const float* x, int64_t n_rows);

/* Parameters / optimizer state in reference order.  For the FV estimator the
 * "params" are the fixed data-term theta (VAEB.py:117-119) and the variational
 * (mu_theta, sigma_theta) pairs are transferred with vaeb_{set,get}_fv_state. */
int vaeb_set_params(vaeb_ctx* ctx, const float* flat, int64_t n);
int vaeb_get_params(vaeb_ctx* ctx, float* flat, int64_t n);
int vaeb_set_adagrad_state(vaeb_ctx* ctx, const float* flat, int64_t n);
int vaeb_get_adagrad_state(vaeb_ctx* ctx, float* flat, int64_t n);
/* FV: mu, sigma and their accumulators, each n = num_params floats. */
int vaeb_set_fv_state(vaeb_ctx* ctx, const float* mu, const float* sigma,
                      const float* acc_mu, const float* acc_sigma, int64_t n);
int vaeb_get_fv_state(vaeb_ctx* ctx, float* mu, float* sigma,
                      float* acc_mu, float* acc_sigma, int64_t n);

/* Noise for the reparameterisation (VAEB.py:41-47).  PHILOX: counter-based normals
 * keyed by (seed, step, global row, l, j), world-size invariant.  HOST: the caller
 * pushes eps [L x rows x Z] before each update/validate chunk (parity mode). */
int vaeb_set_eps_mode(vaeb_ctx* ctx, int32_t mode, uint64_t seed);
int vaeb_push_eps(vaeb_ctx* ctx, const float* eps, int64_t rows, int32_t L);
/* VAEB_EST_FVS in host eps mode: the standard normals zeta [P] (arena order) of the next
 * step's weight sample theta~ = mu + |sigma| zeta (Philox mode draws them on device). */
int vaeb_push_fv_noise(vaeb_ctx* ctx, const float* zeta, int64_t n);
int vaeb_set_step(vaeb_ctx* ctx, int64_t step);   /* Philox step counter */

/* One SGVB step on the contiguous minibatch `batch_index` (VAEB.py:413), synchronous
 * like the reference: writes SGVB / B_global to *out_elbo_per_row. */
int vaeb_update(vaeb_ctx* ctx, int32_t batch_index, float* out_elbo_per_row);
/* Throughput mode: enqueue one step, no host sync.  The ELBO stays on device and is
 * accumulated; read (and reset) the epoch mean with vaeb_epoch_elbo. */
int vaeb_update_async(vaeb_ctx* ctx, int32_t batch_index);
/* Enqueue a whole list of steps (an epoch's batch order) with one call. */
int vaeb_update_many(vaeb_ctx* ctx, const int32_t* batch_indices, int32_t n);
int vaeb_epoch_elbo(vaeb_ctx* ctx, double* out_sum, int64_t* out_steps);
int vaeb_synchronize(vaeb_ctx* ctx);

/* Forward-only SGVB sum over n rows of host x (VAEB.py:418-422). */
int vaeb_validate(vaeb_ctx* ctx, const float* x, int64_t n, double* out_sum);
/* Decoder means y for host x with z = mu (n_samples <= 0 branch of VAEB.reconstruct,
 * VAEB.py:267-270): writes [n x D]. */
int vaeb_reconstruct(vaeb_ctx* ctx, const float* x, int64_t n, float* out_y);
/* VAEB.reconstruct(x, n_samples) (VAEB.py:267-300): n_samples <= 0 as vaeb_reconstruct;
 * otherwise the decoder output averaged over n_samples posterior draws z = mu + exp(lv/2) eps
 * (Philox validation streams 1..n_samples, or in host eps mode rows [s*n, (s+1)*n) of the
 * pushed eps, which must hold n * n_samples rows).  Writes [n x D]. */
int vaeb_reconstruct_sampled(vaeb_ctx* ctx, const float* x, int64_t n, int32_t n_samples, float* out_y);
/* As vaeb_reconstruct_sampled, plus (Gaussian decoder, fp32 contexts; NULL to skip) the
 * decoder's log-sigma head hd W6 + b6 averaged over the same samples (VAEB.py:275-290): the
 * reference's closing draw is y + exp(out_lv) * N(0, 1) per pixel (VAEB.py:293-297). */
int vaeb_reconstruct_full(vaeb_ctx* ctx, const float* x, int64_t n, int32_t n_samples, float* out_y,
                          float* out_lv);
/* The decoder from given latents (freyFace.py:173-187 `image(z)`, compiled as `freyFace` at
 * :237-245): z [n x Z] -> mean [n x D] (sigmoid(tanh(z W1 + b1) W2 + b2)) and, for the Gaussian
 * decoder, the log-sigma head [n x D] (out_lv; NULL to skip).  fp32 contexts. */
int vaeb_decode(vaeb_ctx* ctx, const float* z, int64_t n, float* out_mu, float* out_lv);

/* Data parallel (one ctx per rank): the library owns an RCCL communicator; the 128-byte
 * unique id is produced on rank 0 and broadcast by the host (e.g. torch.distributed). */
int vaeb_comm_unique_id(uint8_t out_id[128]);
int vaeb_comm_init(vaeb_ctx* ctx, const uint8_t id[128], int32_t rank, int32_t world);
/* Ranks in the context's communicator (ncclCommCount); 1 without a communicator. */
int vaeb_comm_count(vaeb_ctx* ctx, int32_t* out_world);

/* Device-resident validation set (VAEB.validate(x_valid) once per epoch, VAEB.py:582):
 * uploaded once; vaeb_validate_resident then evaluates this rank's contiguous share of
 * the rows (all rows without a communicator) with no host round trip between device
 * chunks and, with a communicator, all-reduces the SGVB sum over the ranks.  Noise rows
 * are keyed by the GLOBAL row (Philox), or read from the pushed eps (host mode: eps for
 * all n rows, global row order), so the result does not depend on the world size. */
int vaeb_set_valid_data(vaeb_ctx* ctx, const float* x, int64_t n_rows);
int vaeb_validate_resident(vaeb_ctx* ctx, double* out_sum);

/* Philox step counter (the number of noise draws so far), for checkpoints. */
int vaeb_get_step(vaeb_ctx* ctx, int64_t* step);

/* Native checkpoint (SURVEY 5 "checkpoint / resume"; the reference's VAEB.save keeps theta
 * only, VAEB.py:189-203, so a resumed run restarts Adagrad): one file holding the model
 * shape, theta, the Adagrad accumulators, the Philox seed / step and (FV / FVS) the
 * variational state.  A context loaded from it continues bit-identically to the run that
 * wrote it.  Loading checks that the file's D, H, Z, L, decoder and estimator match.
 * With a sharded data-parallel communicator (world > 1) saving is a collective: every rank
 * calls it (the Adagrad shards are all-gathered first); a rank passing path == NULL joins the
 * gather and writes nothing (rank 0 writes the file); NULL on a context without such a
 * communicator is VAEB_ERR_ARG. */
int vaeb_checkpoint_save(vaeb_ctx* ctx, const char* path);
int vaeb_checkpoint_load(vaeb_ctx* ctx, const char* path);

/* Introspection for parity tests: last step's data gradients (reference order, before
 * the prior) and named device activations ("h","mu","lv","z","hd","dA2","dA3",...). */
int vaeb_get_grads(vaeb_ctx* ctx, float* flat, int64_t n);
int vaeb_get_activation(vaeb_ctx* ctx, const char* name, float* out, int64_t n);

/* ------------------------------------------------------------------------------------------
 * degenerate-vae deterministic autoencoder (/root/reference/degenerate-vae/ae.py:41-117):
 * encoder MLP -> linear latent Z -> decoder MLP -> Bernoulli (otype "binary") or Gaussian
 * ("cont") output, logjoint = loglik + N(0, s2) prior on theta + N(0, 1) prior on Z, AdaGrad.
 * Parameters are flat float32 in the reference's theta order (ae.py:51,56,64,72):
 *   Wenc0..Wenc{n_enc-1}, benc0.., Wz, bz, Wdec0.., bdec0.., then Wout, bout (binary) or
 *   Wmu, Wlogs2, bmu, blogs2 (cont); W row-major [in x out].
 * ------------------------------------------------------------------------------------------ */
#define VAEB_AE_MAX_LAYERS 8
enum vaeb_ae_otype { VAEB_AE_BINARY = 0, VAEB_AE_CONT = 1 };   /* ae.py:58 / :65 */
enum vaeb_act      { VAEB_ACT_TANH = 0, VAEB_ACT_SIGMOID = 1, VAEB_ACT_RELU = 2 };   /* f, ae.py:41 */

typedef struct vaeb_ae_config {
    int32_t Dobs;                         /* observation size                                */
    int32_t n_enc;                        /* len(Denc) >= 1                                  */
    int32_t Denc[VAEB_AE_MAX_LAYERS];     /* encoder hidden sizes                            */
    int32_t Dz;                           /* latent size                                     */
    int32_t n_dec;                        /* len(Ddec) >= 1                                  */
    int32_t Ddec[VAEB_AE_MAX_LAYERS];     /* decoder hidden sizes                            */
    int32_t otype;                        /* enum vaeb_ae_otype                              */
    int32_t act;                          /* enum vaeb_act                                   */
    float   s2;                           /* prior variance on theta (ae.py:41, default 1.0) */
    float   eta;                          /* AdaGrad learning rate (infalg.py:144)           */
    int32_t max_batch;                    /* largest idx list / predict chunk                */
    int32_t device;
    int32_t reserved[4];
} vaeb_ae_config;

typedef struct vaeb_ae vaeb_ae;

int vaeb_ae_create(const vaeb_ae_config* cfg, vaeb_ae** out);   /* ConstructAE (ae.py:41)    */
int vaeb_ae_destroy(vaeb_ae* ae);
int vaeb_ae_num_params(const vaeb_ae* ae, int64_t* n);
int vaeb_ae_set_data(vaeb_ae* ae, const float* x, int64_t n_rows);   /* Xtr (ae.py:87)        */
int vaeb_ae_set_params(vaeb_ae* ae, const float* flat, int64_t n);
int vaeb_ae_get_params(vaeb_ae* ae, float* flat, int64_t n);
int vaeb_ae_set_adagrad_state(vaeb_ae* ae, const float* flat, int64_t n);
int vaeb_ae_get_adagrad_state(vaeb_ae* ae, float* flat, int64_t n);
/* train(idx) (ae.py:82-89): one AdaGrad step on rows Xtr[idx]; writes loglik / n. */
int vaeb_ae_train(vaeb_ae* ae, const int32_t* idx, int32_t n, float* out_loglik_per_row);
/* An epoch of train() calls on consecutive `batch`-sized slices of idx, the last partial
 * slice kept (ae.py:145-151); out[j] = train's value for slice j.  One host sync. */
int vaeb_ae_train_many(vaeb_ae* ae, const int32_t* idx, int32_t n, int32_t batch, float* out);
int vaeb_ae_reconstruct(vaeb_ae* ae, const float* x, int64_t n, float* out);   /* ae.py:92-98  */
int vaeb_ae_encode(vaeb_ae* ae, const float* x, int64_t n, float* z_out);      /* ae.py:101-107 */
int vaeb_ae_decode(vaeb_ae* ae, const float* z, int64_t n, float* out);        /* ae.py:110-116 */

#ifdef __cplusplus
}
#endif
#endif /* VAEB_HIP_H */
