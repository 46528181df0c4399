// vaeb_hip.hip -- C ABI (include/vaeb_hip.h) over the gfx950 SGVB step kernels.
//
// One context = one GPU (one rank).  All state lives in device memory owned here:
// a flat parameter arena in the reference order (VAEB.py:111-115) with matching
// Adagrad-accumulator and gradient arenas, the device-resident training set
// (th.shared x_train, VAEB.py:184), activation/delta buffers, and a small control
// block (batch order, cursor, Philox step, ELBO accumulators) so a step needs no host
// round trip and can be replayed as a hipGraph.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <type_traits>

#include "../../include/vaeb_diag.h"   // includes vaeb_hip.h
#include "hfuse.hpp"
#include "latent.hpp"
#include "latent_bwd.hpp"
#include "h16_engines.hpp"
#include "ae_mlp.hpp"

using namespace vaeb;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (void)hipGetLastError(); /* a failed call must not resurface at the next launch */ \
            return fail(VAEB_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                               \
        }                                                                                  \
    } while (0)

#define CHECK_LAUNCH()                                                                     \
    do {                                                                                   \
        hipError_t e_ = hipGetLastError();                                                 \
        if (e_ != hipSuccess)                                                              \
            return fail(VAEB_ERR_HIP, "kernel launch failed: %s (%s:%d)",                  \
                        hipGetErrorString(e_), __FILE__, __LINE__);                        \
    } while (0)

inline int r16(int x) { return (x + 15) & ~15; }
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

template <class T>
int dalloc(T** p, size_t n) {
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void**)p, n * sizeof(T));
    if (e != hipSuccess) return fail(VAEB_ERR_NOMEM, "hipMalloc(%zu) failed: %s", n * sizeof(T), hipGetErrorString(e));
    // the zero fill runs on the null stream, which does not order against the contexts'
    // non-blocking streams: wait for it here, or a kernel enqueued next on a context stream can
    // run before (or beside) the fill and have its stores overwritten with zeros
    e = hipMemset(*p, 0, n * sizeof(T));
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) return fail(VAEB_ERR_HIP, "zero fill of %zu bytes: %s", n * sizeof(T), hipGetErrorString(e));
    return 0;
}

// Control block layout (ints): [0] cursor, [1] resolved batch, [2..] batch order.
constexpr int kFvParts = 1024;   // FV stream grid (one thetaPrior partial per block)
constexpr int kGraphSteps = 32;  // the longest replayed graph
constexpr int kMaxProfKernels = 24;
constexpr int kDbgWG = 1024;      // diagnostics: stamp slots per launch (workgroups)

const char* kKernelNames[] = {"p1_enc", "p2_heads", "p3_dechid", "p4_decout", "p5_dhd_w2", "p6_dz",
                              "p7_dh", "p8_wgrad_w3w45", "allreduce", "adagrad", "fv_update", "elbo",
                              "p23_heads_dechid", "p67_dz_dh_w1", "p8_wgrad_w2", "p8_wgrad_w1",
                              "p1_enc_latent", "p4_decout_z",
                              // bf16 engine (step_bf16.hpp), ids 18..34
                              "bf_enc", "bf_heads", "bf_latent", "bf_dechid", "bf_decout", "bf_dhd", "bf_dW26",
                              "bf_dz", "bf_dW1", "bf_dW1_opt", "bf_latent_bwd", "bf_dh", "bf_dW45", "bf_dW45_opt",
                              "bf_dW3", "bf_bias_elbo", "bf_adagrad_dp",
                              // weight-sampling full-variational extension, ids 35..38
                              "unused35", "unused36", "fvs_sample", "fvs_update",
                              // folded latent backward (latent_bwd.hpp), ids 39..40
                              "p5_dhd_dz_w2", "p8_wgrad_w3w45w1",
                              // bf16 engine: dhd and dW2 (| dW6) in one grid, id 41
                              "bf_dhd_dW26",
                              // deferred dW2 (round 4): the encoder launch carries the previous
                              // step's dW2 tiles; the dhd launch has none, ids 42..43
                              "p1_enc_latent_w2", "p5_dhd_dz"};

}  // namespace

struct vaeb_ctx {
    vaeb_config c{};
    hipStream_t s = nullptr;   // every step launch goes to this one stream
    int64_t P = 0;
    int nparams = 0;
    int64_t off[12] = {};   // arena offsets, reference order
    // arenas
    float* theta2[2] = {nullptr, nullptr};   // ping-pong parameter arenas
    int par = 0;                              // arena holding the current parameters
    float *acc = nullptr, *grad = nullptr;
    float *fvmu = nullptr, *fvsg = nullptr, *fvam = nullptr, *fvas = nullptr, *fv_part = nullptr;
    float* fvzeta = nullptr;   // VAEB_EST_FVS host-mode weight noise [P]
    // data
    float* data = nullptr;
    int64_t nrows = 0;
    float* xeval = nullptr;
    float* xval = nullptr;        // resident validation set (vaeb_set_valid_data; bf16: bf.xval)
    int64_t nval = 0;
    // control
    int* ictl = nullptr;          // cursor, cur_batch, order[kOrderCap], next (tile_engine.hpp)
    int64_t* step = nullptr;
    float* elbo_out = nullptr;
    double* epoch = nullptr;      // [2] of the control block blk (kernels_aux.hpp kBlk*)
    uint64_t* blk = nullptr;      // epoch [2], status, elbo_out, fixed-point guard word, acc_ml, acc_dz
    double* eval_acc = nullptr;   // [2]
    // noise
    int eps_mode = VAEB_EPS_PHILOX;
    uint64_t seed = 10;
    float* eps_in = nullptr;
    int64_t eps_in_cap = 0, eps_rows = 0;
    // activations
    int cap = 0;                  // padded row capacity (per l plane)
    float *h = nullptr, *mu = nullptr, *lv = nullptr, *eps = nullptr, *z = nullptr, *hd = nullptr,
          *y = nullptr, *dA2 = nullptr, *dA6 = nullptr, *dA1 = nullptr, *dZ = nullptr,
          *dMuLv = nullptr, *dA3 = nullptr, *kl_part = nullptr, *lp_part = nullptr;
    float* yacc = nullptr;        // sampled reconstruction sum (allocated on first use)
    float *slab_ml = nullptr, *slab_dz = nullptr;  // folded-latent partial slabs (latent.hpp)
    int *cnt_ml = nullptr, *cnt_dz = nullptr;      // their per-row-block arrival counters
    uint64_t *acc_ml = nullptr, *acc_dz = nullptr; // atomic hand-off accumulators (zeroed)
    // host staging (pinned)
    int* h_ctl = nullptr;
    float* h_elbo = nullptr;
    double* h_d2 = nullptr;
    float* h_out = nullptr;       // mapped host [SGVB / B, flags] every training step's last kernel writes
    bool async_pending = false;   // steps enqueued by vaeb_update_many / _async not yet synchronised
    hipEvent_t ctl_ev = nullptr;
    // graphs
    hipGraphExec_t gN[2][kGraphSteps + 1] = {};  // gN[p][n]: n steps from arena p (run_steps)
    bool graph_failed = false;
    std::string graph_err;        // why the capture failed (vaeb_graph_status)
    // comm
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    hipStream_t s3 = nullptr;     // bf16 engine: dW2 (| dW6) + Adagrad forked beside the backward chain
    hipEvent_t fk_ev[4] = {};     // fork after dhd, s3's work done, [dMu | dLv] ready, ELBO partials
    int bf_thin = 3;              // VAEB_BF_THIN mask: 1 heads, 2 dz on thin_bf16.hpp (0: split-K + latent kernels)
    bool bf_fork = true;          // VAEB_BF_FORK=0: dW2 in the dhd grid (bf_fuse) or after it
    int bf_dzfuse = 1;            // VAEB_BF_DZFUSE=0: dz + latent backward on the thin launch instead of in the forked dhd
    int bf_dtt = 1;               // VAEB_BF_DTT=0: dhd / dh on A W (EpiDTanh) instead of the transpose (EpiDTanhT)
    hipStream_t s2 = nullptr;     // DP: the gradient buckets' all-reduces and their Adagrad
    hipEvent_t dp_ev[3] = {};     // fork after dW2, bucket A reduced, bucket A updated
    bool dp_overlap = false;      // bucket A on s2 (bf16 engine; VAEB_DP_OVERLAP=0/1 overrides)
    bool dp_shard = false;        // reduce-scatter -> this rank's shard of Adagrad -> all-gather (world > 1)
    bool fold_bwd = true;         // Z <= 32: latent backward folded into the dhd launch (VAEB_FOLD_BWD=0: P67)
    // slab form of the folded backward (fan-in > 16): the dZ slab sum and [dMu | dLv] by
    // reducer workgroups of the LAST launch (kernels_aux.hpp LatRed) instead of a ticket and
    // a last-arriver reducer in the dhd launch.  VAEB_BWD_DEFER=0: the ticketed form.
    bool bwd_defer = true;
    // the deferred dW2: dW2 (| dW6) + Adagrad of step t run in step t+1's encoder launch, on
    // the CUs the encoder leaves idle (latent.hpp enc_latent16_w2_kernel), so the dhd launch
    // holds the dhd tiles alone; host reads of the state flush a pending one first (w2_flush).
    // fp32 LB / LA, no communicator, 16-wave encoder, the latent backward deferred too (ho_dz 2:
    // dw2_deferred).  VAEB_DW2_DEFER=0: dW2 in the dhd launch.
    bool dw2_defer = true;
    int* w2pend = nullptr;        // device: 1 = a step's dW2 is pending (set by its dhd launch)
    bool w2_dirty = false;        // host: a step was enqueued since the last flush
    bool w2_graph = false;        // host: the captured graphs hold deferred-dW2 steps (run_steps sets w2_dirty)
    int atomic_ho = 1;            // folded latent hand-offs: 1 by fan-in (ho_mode), 0 slabs
    int enc_red = -1;             // encoder slabs summed by the decoder launch: -1 auto, VAEB_ENC_RED=0|1
    // update_many's order upload held back until the eager first step's first launch is out
    // (order_hook): the upload kernel then runs behind the encoder instead of ahead of it
    bool order_pending = false;
    OrderArg order_pend;
    // profiling
    hipEvent_t pev[kMaxProfKernels + 1] = {};
    int prof_n = 0, prof_reps = 1;
    std::vector<int> prof_ids;
    // diagnostics timeline (vaeb_debug_timeline)
    uint64_t* dbg = nullptr;
    int dbg_slot = 0;
    // bf16 large-batch engine (step_bf16.hpp); off for dtype == VAEB_DTYPE_F32
    h16c::BfState bf;
};

namespace {

bool gaussian(const vaeb_ctx* c) { return c->c.decoder == VAEB_DEC_GAUSSIAN; }

// The parameter arena in reference order W3 W4 W5 W1 W2 [W6] b3 b4 b5 b1 b2 [b6]
// (VAEB.py:74-104): c->off, c->nparams, c->P from the config alone (no device call).
void set_arena_layout(vaeb_ctx* c) {
    const int64_t D = c->c.D, H = c->c.H, Z = c->c.Z;
    std::vector<int64_t> sz = {D * H, H * Z, H * Z, Z * H, H * D};
    if (gaussian(c)) sz.push_back(H * D);
    sz.insert(sz.end(), {H, Z, Z, H, D});
    if (gaussian(c)) sz.push_back(D);
    c->nparams = (int)sz.size();
    int64_t o = 0;
    for (int i = 0; i < c->nparams; ++i) { c->off[i] = o; o += sz[i]; }
    c->P = o;
}

uint64_t* next_dbg(vaeb_ctx* c) { return c->dbg ? c->dbg + (size_t)(c->dbg_slot++) * kDbgWG * 8 : nullptr; }

int order_hook(vaeb_ctx* c);

StepArgs make_args(vaeb_ctx* c, int par, int Mb, int mode, const float* xbase, bool train) {
    StepArgs a{};
    const vaeb_config& g = c->c;
    a.D = g.D; a.H = g.H; a.Z = g.Z; a.L = g.L;
    a.Mb = Mb; a.Mbp = r16(Mb); a.Me = g.L * a.Mbp;
    a.dec = g.decoder; a.est = g.estimator == VAEB_EST_FVS ? VAEB_EST_LB : g.estimator; a.mode = mode;
    a.sc = (g.objective == VAEB_OBJ_MEAN_MAP) ? 1.0f / (float)g.B_global : 1.0f;
    const float* t = c->theta2[par];
    const bool gs = gaussian(c);
    // reference order: W3,W4,W5,W1,W2,(W6),b3,b4,b5,b1,b2,(b6)
    a.W3 = t + c->off[0]; a.W4 = t + c->off[1]; a.W5 = t + c->off[2]; a.W1 = t + c->off[3];
    a.W2 = t + c->off[4];
    const int bo = gs ? 6 : 5;
    a.W6 = gs ? t + c->off[5] : nullptr;
    a.b3 = t + c->off[bo + 0]; a.b4 = t + c->off[bo + 1]; a.b5 = t + c->off[bo + 2];
    a.b1 = t + c->off[bo + 3]; a.b2 = t + c->off[bo + 4];
    a.b6 = gs ? t + c->off[bo + 5] : nullptr;
    a.xbase = xbase;
    if (train) {
        // this rank's rows of global minibatch b start at row b * B_global + row_offset
        a.xbase = xbase + (int64_t)g.row_offset * g.D;
        a.order = c->ictl + kCtlOrder;
        a.cursor = c->ictl;
        a.cur_batch = c->ictl + 1;
        a.batch_stride = (int64_t)g.B_global * g.D;
        a.row_base_mul = g.B_global;
        a.row_base_add = g.row_offset;
        a.domain = 0;
    } else {
        a.order = nullptr; a.cursor = nullptr; a.cur_batch = c->ictl + 1;
        a.batch_stride = 0; a.row_base_mul = 0; a.row_base_add = 0;
        a.domain = 1;
    }
    a.eps_mode = (mode == MODE_RECON) ? 2 : (c->eps_mode == VAEB_EPS_HOST ? 1 : 0);
    a.seed = c->seed;
    a.step = c->step;
    a.eps_in = c->eps_in;
    a.eps_in_ld = c->eps_rows;
    a.h = c->h; a.mu = c->mu; a.lv = c->lv; a.eps = c->eps; a.z = c->z; a.hd = c->hd; a.y = c->y;
    a.dA2 = c->dA2; a.dA6 = c->dA6; a.dA1 = c->dA1; a.dZ = c->dZ; a.dMuLv = c->dMuLv; a.dA3 = c->dA3;
    a.kl_part = c->kl_part; a.la_part = c->kl_part; a.lp_part = c->lp_part;
    a.nctZ = cdiv(g.Z, 16);
    a.nctD = cdiv(g.D, 16);
    a.slab_ml = c->slab_ml; a.slab_dz = c->slab_dz; a.cnt_ml = c->cnt_ml; a.cnt_dz = c->cnt_dz;
    a.acc_ml = c->acc_ml; a.acc_dz = c->acc_dz;
    return a;
}

template <int WM, int WN, int KS, int NB, int GCH, class P>
void launch_tile(hipStream_t s, const P& p) {
    dim3 grid(cdiv(p.M, 16 * WM), cdiv(p.N, 16 * WN));
    hipLaunchKernelGGL((tile_kernel<WM, WN, KS, NB, GCH, P>), grid, dim3(64 * WM * WN * KS), 0, s, p);
}

// Big-K phases: 8 waves split K; a wave's chunks go in flight together (GCH per trip).
template <int NB, class P>
void launch_bigk(hipStream_t s, const P& p) {
    const int per_wave = cdiv(cdiv(p.K, 16), 8);
    if (per_wave <= 4) launch_tile<1, 1, 8, NB, 4>(s, p);
    else launch_tile<1, 1, 8, NB, 8>(s, p);
}

bool fused_latent(const vaeb_ctx* c) { return c->c.Z <= 32; }
// Weight-gradient tile widths (columns; rows are kWT = 64).  Narrower tiles mean more
// workgroups, each streaming fewer theta / accumulator / panel bytes through its CU: at
// MNIST-20, 64 -> 32 wide took the dW2 launch 11.7 -> 9.5 us and the dW3 | dW45 launch
// 10.9 -> 8.1 us; 16 wide takes the latter to 7.5 us but the dW2 launch (beside 224 dhd
// tiles) back up to 11.1 us.
constexpr int kWTJ_P5 = 32;    // dW2 (| dW6), beside the dhd tiles (64 wide: 40.1 vs 38.8 us per step)
constexpr int kW3TS = 1;       // 16-column groups per tile of the last launch (dW3 | dW45 | dW1; 2: 40.1 vs 38.8)
constexpr int kWTJ_P67 = 16;   // dW1, beside the dz / dh phase
constexpr int kWTJ_W = 16;     // standalone launches: dW3 | dW45 (+ ELBO), non-fused dW1
constexpr int kDzSplit = 8;    // P67 column splits per row block (fused.hpp dz_dh_body)

// The deferred dW2's launch arguments (the previous step's dW2 (| dW6) group; vaeb_ctx::dw2_defer)
struct W2Launch {
    WGradArgs w;
    bool vec;
    const int* pend;
};

// The folded latent hand-offs: counted fixed-point atomics (latent.hpp fx_*) or slabs +
// ticket + reducer.  The returning adds to one accumulator serialise at the memory side, so
// the atomic form wins only at a small fan-in (contributors per element): Frey 560-200-2
// (13 column tiles) 38.5 -> 32.2 us per step; MNIST 784-500-20 (32 column tiles) 44.5 ->
// 49.3 us.  Forward fan-in: the H column tiles; backward: H column tiles x L planes.
// (A third form -- the same adds without return + the slab protocol's ticket, the last
// arriver reading each sum with one exchange -- measured slower than both, MNIST 53.6 us,
// Frey 35.0 us, and was removed in round 3.)  VAEB_ATOMIC_HO=0 forces the slabs.
int ho_mode(const vaeb_ctx* c, int fan_in) {
    if (c->atomic_ho == 0) return 0;
    return fan_in <= kFxMaxFanIn ? 1 : 0;   // the count field holds <= 16 contributors (latent.hpp)
}
int ho_ml(const vaeb_ctx* c, int ct) { return ho_mode(c, cdiv(c->c.H, 16 * ct)); }
bool dw2_deferrable(const vaeb_ctx* c);
// backward: 1 atomic, else 2 (deferred to the last launch's reducers, VAEB_BWD_DEFER) or 0
// (ticket).  (Round 5's form 3 -- two dA1 column tiles per 1024-thread dhd workgroup so MNIST's
// fan-in fits the counted atomics -- measured 39.4 vs 34.4 us per step and was removed in round 6.)
int ho_dz(const vaeb_ctx* c) {
    const int m = ho_mode(c, cdiv(c->c.H, 16) * c->c.L);
    return m == 0 && c->bwd_defer ? 2 : m;
}

// Measurement brackets: mark(id) records an event before launch slot `id`.  With
// reps > 1 (vaeb_profile_steps) every launch of the step is issued `reps` times back to
// back inside its bracket, so bracket time / reps is a kernel's duration plus one
// same-kernel launch gap, free of the event packets' own cost.
#define REP(pr) for (int r_ = 0; r_ < (pr).reps; ++r_)
struct Prof {
    vaeb_ctx* c;
    bool on;
    int reps = 1;
    int k = 0;
    void mark(int id) {
        if (!on) return;
        hipEventRecord(c->pev[k], c->s);
        if (k < (int)c->prof_ids.size()) c->prof_ids[k] = id; else c->prof_ids.push_back(id);
        ++k;
    }
};

ElboArgs base_elbo(vaeb_ctx* c, const StepArgs& a) {
    ElboArgs e{};
    e.lp_part = c->lp_part; e.n_lp = (int64_t)a.Me * a.nctD;
    e.kl_part = c->kl_part;
    e.n_kl = (int64_t)(c->c.estimator == VAEB_EST_LA ? a.Me : a.Mbp) * a.nctZ;
    e.L = c->c.L; e.est = c->c.estimator;
    e.data_mul = 1.0;
    e.inv_bglob = 1.0 / (double)c->c.B_global;
    return e;
}

template <int NB, bool V1, int AT>
void launch_decout_zv(hipStream_t s, dim3 grid, const StepArgs& a, int ct) {
    if (NB == 1 && ct == 2) {   // two column tiles per workgroup
        switch ((a.Z + 3) / 4) {
            case 1: hipLaunchKernelGGL((decout_z2_kernel<1, V1, AT>), grid, dim3(512), 0, s, a); break;
            case 2: hipLaunchKernelGGL((decout_z2_kernel<2, V1, AT>), grid, dim3(512), 0, s, a); break;
            case 3: case 4: hipLaunchKernelGGL((decout_z2_kernel<4, V1, AT>), grid, dim3(512), 0, s, a); break;
            case 5: hipLaunchKernelGGL((decout_z2_kernel<5, V1, AT>), grid, dim3(512), 0, s, a); break;
            default: hipLaunchKernelGGL((decout_z2_kernel<8, V1, AT>), grid, dim3(512), 0, s, a); break;
        }
        return;
    }
    switch ((a.Z + 3) / 4) {
        case 1: hipLaunchKernelGGL((decout_z_kernel<NB, 1, V1, AT>), grid, dim3(512), 0, s, a); break;
        case 2: hipLaunchKernelGGL((decout_z_kernel<NB, 2, V1, AT>), grid, dim3(512), 0, s, a); break;
        case 3: case 4: hipLaunchKernelGGL((decout_z_kernel<NB, 4, V1, AT>), grid, dim3(512), 0, s, a); break;
        case 5: hipLaunchKernelGGL((decout_z_kernel<NB, 5, V1, AT>), grid, dim3(512), 0, s, a); break;
        default: hipLaunchKernelGGL((decout_z_kernel<NB, 8, V1, AT>), grid, dim3(512), 0, s, a); break;
    }
}
template <int NB, int AT>
void launch_decout_z(hipStream_t s, dim3 grid, const StepArgs& a, int ct = 1) {
    auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    if ((a.H & 3) == 0 && al(a.W1) && al(a.b1)) launch_decout_zv<NB, true, AT>(s, grid, a, ct);
    else launch_decout_zv<NB, false, AT>(s, grid, a, ct);
}

// dhd_dz_wgrad_kernel at compile-time NCT (latent col tiles), GCH, load width, AT
template <int TS, int HO>
void launch_dhd_dz(hipStream_t s, dim3 grid, const PDhdT<true>& p5, const PDhdT<false>& p5s, const WGradArgs& w,
                   int ntile, int gx, bool vec, bool deep, DhdAux pend) {
    if (p5.a.Z <= 16) {
        if (deep) {
            if (vec) hipLaunchKernelGGL((dhd_dz_wgrad_kernel<1, 8, true, TS, HO>), grid, dim3(512), 0, s, p5, w, ntile, gx, pend);
            else hipLaunchKernelGGL((dhd_dz_wgrad_kernel<1, 8, false, TS, HO>), grid, dim3(512), 0, s, p5s, w, ntile, gx, pend);
        } else {
            if (vec) hipLaunchKernelGGL((dhd_dz_wgrad_kernel<1, 4, true, TS, HO>), grid, dim3(512), 0, s, p5, w, ntile, gx, pend);
            else hipLaunchKernelGGL((dhd_dz_wgrad_kernel<1, 4, false, TS, HO>), grid, dim3(512), 0, s, p5s, w, ntile, gx, pend);
        }
    } else {
        if (deep) {
            if (vec) hipLaunchKernelGGL((dhd_dz_wgrad_kernel<2, 8, true, TS, HO>), grid, dim3(512), 0, s, p5, w, ntile, gx, pend);
            else hipLaunchKernelGGL((dhd_dz_wgrad_kernel<2, 8, false, TS, HO>), grid, dim3(512), 0, s, p5s, w, ntile, gx, pend);
        } else {
            if (vec) hipLaunchKernelGGL((dhd_dz_wgrad_kernel<2, 4, true, TS, HO>), grid, dim3(512), 0, s, p5, w, ntile, gx, pend);
            else hipLaunchKernelGGL((dhd_dz_wgrad_kernel<2, 4, false, TS, HO>), grid, dim3(512), 0, s, p5s, w, ntile, gx, pend);
        }
    }
}

// enc_latent_kernel / enc_latent_fv_kernel at compile-time NCT (latent col tiles), GCH
// (main-loop chunk group), AT (atomic hand-off)
template <int HO, int CT>
void launch_enc_latent_ct(hipStream_t s, dim3 g1, const StepArgs& a, const FvFold& fvf, bool deep) {
    if (fvf.rows > 0) {
        if (a.Z <= 16) {
            if (deep) hipLaunchKernelGGL((enc_latent_fv_kernel<1, 8, HO, CT>), g1, dim3(512), 0, s, a, fvf);
            else hipLaunchKernelGGL((enc_latent_fv_kernel<1, 4, HO, CT>), g1, dim3(512), 0, s, a, fvf);
        } else {
            if (deep) hipLaunchKernelGGL((enc_latent_fv_kernel<2, 8, HO, CT>), g1, dim3(512), 0, s, a, fvf);
            else hipLaunchKernelGGL((enc_latent_fv_kernel<2, 4, HO, CT>), g1, dim3(512), 0, s, a, fvf);
        }
    } else if (a.Z <= 16) {
        if (deep) hipLaunchKernelGGL((enc_latent_kernel<1, 8, HO, CT>), g1, dim3(512), 0, s, a);
        else hipLaunchKernelGGL((enc_latent_kernel<1, 4, HO, CT>), g1, dim3(512), 0, s, a);
    } else {
        if (deep) hipLaunchKernelGGL((enc_latent_kernel<2, 8, HO, CT>), g1, dim3(512), 0, s, a);
        else hipLaunchKernelGGL((enc_latent_kernel<2, 4, HO, CT>), g1, dim3(512), 0, s, a);
    }
}
// The 16-wave encoder with the deferred dW2 workers (w2: the previous step's dW2 group) in
// ceil(ntile / 2 / (Mbp / 16)) extra grid rows.
template <int HO, int CT>
void launch_enc16_w2(hipStream_t s, dim3 g1, const StepArgs& a, const W2Launch& w2) {
    const int rows = (int)g1.y;
    const dim3 g(g1.x, g1.y + cdiv(cdiv(w2.w.total_wgs, 2), (int)g1.x));
    constexpr int TS = kWTJ_P5 / 16;
    if (a.Z <= 16) {
        if (w2.vec) hipLaunchKernelGGL((enc_latent16_w2_kernel<1, 4, HO, CT, true, TS>), g, dim3(1024), 0, s, a, w2.w, w2.pend, rows);
        else hipLaunchKernelGGL((enc_latent16_w2_kernel<1, 4, HO, CT, false, TS>), g, dim3(1024), 0, s, a, w2.w, w2.pend, rows);
    } else {
        if (w2.vec) hipLaunchKernelGGL((enc_latent16_w2_kernel<2, 4, HO, CT, true, TS>), g, dim3(1024), 0, s, a, w2.w, w2.pend, rows);
        else hipLaunchKernelGGL((enc_latent16_w2_kernel<2, 4, HO, CT, false, TS>), g, dim3(1024), 0, s, a, w2.w, w2.pend, rows);
    }
}

// The slab-only encoder (HO 3: partials summed by the decoder launch, CT = 2, no FV) and the
// atomic hand-off encoder (HO 1, one column tile, no FV) run on 1024-thread workgroups, 16
// waves splitting K (twice the loads in flight per CU): MNIST 38.82 -> 37.87 us/step, Frey
// 29.19 -> 29.01 in round 3's alternating runs (the 512-thread forms' switch, VAEB_ENC16, was
// removed in round 6).  The ticketed reducer (HO 0) and the FV-stream encoder keep 512 threads.
template <int HO>
void launch_enc_latent(hipStream_t s, dim3 g1, const StepArgs& a, const FvFold& fvf, bool deep, int ct,
                       const W2Launch* w2 = nullptr) {
    if constexpr (HO == 3) {
        if (w2) { launch_enc16_w2<HO, 2>(s, g1, a, *w2); return; }
        if (a.Z <= 16) hipLaunchKernelGGL((enc_latent16_kernel<1, 4, HO, 2>), g1, dim3(1024), 0, s, a);
        else hipLaunchKernelGGL((enc_latent16_kernel<2, 4, HO, 2>), g1, dim3(1024), 0, s, a);
        return;
    }
    if (HO == 1 && fvf.rows == 0 && ct == 1) {   // the atomic hand-off on 16 waves
        if constexpr (HO == 1) if (w2) { launch_enc16_w2<1, 1>(s, g1, a, *w2); return; }
        if (a.Z <= 16) hipLaunchKernelGGL((enc_latent16_kernel<1, 4, 1, 1>), g1, dim3(1024), 0, s, a);
        else hipLaunchKernelGGL((enc_latent16_kernel<2, 4, 1, 1>), g1, dim3(1024), 0, s, a);
        return;
    }
    if (ct == 2) launch_enc_latent_ct<HO, 2>(s, g1, a, fvf, deep);
    else launch_enc_latent_ct<HO, 1>(s, g1, a, fvf, deep);
}

// Training minibatches with Z <= 32 fold the latent block into the wide phases
// (latent.hpp); validation / reconstruction chunks keep the per-row-block kernels.
bool folded_latent(const vaeb_ctx* c, const StepArgs& a) {
    return fused_latent(c) && a.domain == 0 && a.Mbp <= r16(c->c.B);   // training rows (domain 0)
}

// Forward phases P1..P4 for any mode.
// The encoder form the folded forward takes for `a` (enqueue_forward): ho (3 slabs summed by
// the decoder, 1 counted atomics, 0 ticket), ct column tiles per workgroup; true when that
// form runs on 16-wave workgroups (enc_latent16_kernel), the one that can carry the deferred dW2.
bool enc_form(const vaeb_ctx* c, const StepArgs& a, const FvFold& fvf, int* ho_out, int* ct_out, bool* red_out) {
    const bool red = (c->enc_red < 0 ? ho_ml(c, 1) == 0 : c->enc_red == 1) && fvf.rows == 0 && cdiv(a.H, 32) <= 32;
    const int ct = (red || fvf.rows > 0) ? 2 : 1;
    // (round 4's HO 4 -- the [mu | lv] partials as exact fixed-point sums read by the decoder,
    // VAEB_ENC_FX -- measured 34.8-35.1 vs 34.4-34.5 us per step and was removed in round 6)
    const int ho = red ? 3 : ho_ml(c, ct);
    if (ho_out) *ho_out = ho;
    if (ct_out) *ct_out = ct;
    if (red_out) *red_out = red;
    return ho == 3 || (ho == 1 && fvf.rows == 0 && ct == 1);
}

int enqueue_forward(vaeb_ctx* c, const StepArgs& a0, Prof& pr, const FvFold& fvf = FvFold{},
                    const W2Launch* w2 = nullptr) {
    hipStream_t s = c->s;
    StepArgs a = a0;
    a.dbg = next_dbg(c);
    if (folded_latent(c, a)) {
        // auto: two column tiles per workgroup when the literal-FV stream shares the launch
        // (FV 27.75 -> 27.4 us: fewer encoder tiles beside the stream blocks), else one
        // (MNIST 44.6 either way, Frey 32.2 vs 34.0 us)
        // VAEB_ENC_RED=1: no hand-off in the encoder launch at all -- its CT = 2 tiles store
        // partial [mu | lv] slabs and end; every decoder workgroup sums its row block's
        // ceil(H / 32) slabs (decout_z_kernel<.., ZM = 2>)
        // auto: where the slab + ticket form would be chosen (fan-in > 16; MNIST 784-500-20
        // 43.8 -> 42.5 us); at a small fan-in the counted atomics stay (Frey 30.8 vs 32.7 us)
        int ho, ct;
        bool red;
        enc_form(c, a, fvf, &ho, &ct, &red);
        const dim3 g1(a.Mbp / 16, cdiv(a.H, 16 * ct) + fvf.rows);
        const bool deep = cdiv(cdiv(a.D, 16), 8) > 4;
        const int at = red ? 2 : (ho == 1 ? 1 : 0);
        pr.mark(w2 ? 42 : 16);
        REP(pr) {
            if (ho == 3) launch_enc_latent<3>(s, g1, a, fvf, deep, ct, w2);
            else if (ho == 1) launch_enc_latent<1>(s, g1, a, fvf, deep, ct, w2);
            else launch_enc_latent<0>(s, g1, a, fvf, deep, ct);
        }
        CHECK_LAUNCH();
        if (int rc = order_hook(c)) return rc;
        a.dbg = next_dbg(c);
        // Bernoulli: two 16-column tiles per workgroup (decout_z2_kernel; one tile: 42.0 vs
        // 39.4 us per step in round 3, its switch VAEB_DECOUT_CT removed in round 6)
        const int dct = gaussian(c) ? 1 : 2;
        const dim3 g4(a.Me / 16, cdiv(a.D, 16 * dct));
        pr.mark(17);
        REP(pr) {
            if (gaussian(c)) {
                if (at == 2) launch_decout_z<2, 2>(s, g4, a);
                else if (at == 1) launch_decout_z<2, 1>(s, g4, a);
                else launch_decout_z<2, 0>(s, g4, a);
            } else {
                if (at == 2) launch_decout_z<1, 2>(s, g4, a, dct);
                else if (at == 1) launch_decout_z<1, 1>(s, g4, a, dct);
                else launch_decout_z<1, 0>(s, g4, a, dct);
            }
        }
        CHECK_LAUNCH();
        return 0;
    }
    pr.mark(0);
    REP(pr) launch_bigk<1>(s, PEnc{a, nullptr, a.Mbp, a.H, a.D});
    CHECK_LAUNCH();
    a.dbg = next_dbg(c);
    if (fused_latent(c)) {
        pr.mark(12);
        REP(pr) {
            if (a.Z <= 16) hipLaunchKernelGGL(heads_dechid_kernel<1>, dim3(a.Mbp / 16), dim3(512), 0, s, a);
            else hipLaunchKernelGGL(heads_dechid_kernel<2>, dim3(a.Mbp / 16), dim3(512), 0, s, a);
        }
        CHECK_LAUNCH();
    } else {
        pr.mark(1);
        REP(pr) launch_tile<1, 1, 4, 2, 8>(s, PHeads{a, a.Mbp, a.Z, a.H});
        CHECK_LAUNCH();
        pr.mark(2);
        REP(pr) launch_tile<1, 4, 1, 1, 8>(s, PDecHid{a, a.Me, a.H, a.Z});
        CHECK_LAUNCH();
    }
    a.dbg = next_dbg(c);
    pr.mark(3);
    REP(pr) {
        if (gaussian(c)) launch_bigk<2>(s, PDecOut{a, nullptr, a.Me, a.D, a.H});
        else launch_bigk<1>(s, PDecOut{a, nullptr, a.Me, a.D, a.H});
    }
    CHECK_LAUNCH();
    return 0;
}

OptArgs make_opt(vaeb_ctx* c, int par, bool update, bool store) {
    OptArgs o{};
    o.theta_in = c->theta2[par];
    o.theta_out = c->theta2[par ^ 1];
    o.acc = c->acc; o.grad = c->grad;
    o.lr = c->c.lr; o.eps = c->c.adagrad_eps;
    const bool mean = c->c.objective == VAEB_OBJ_MEAN_MAP;
    o.prior = mean ? 0.f : 1.f;
    o.decay = mean ? c->c.lr * c->c.adagrad_eps : 0.f;
    o.update = update ? 1 : 0;
    o.store_grad = store ? 1 : 0;
    return o;
}

// 16-byte dhd operand loads (PDhdT<true>): D % 4 == 0 and 16-byte aligned dA2 / W2 (the
// Gaussian halves dA6 / W6 then are too: they sit a multiple of 4 elements further).
bool dhd_vec(const StepArgs& a) {
    auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    return (a.D & 3) == 0 && al(a.dA2) && al(a.W2);
}


void set_head(WGradArgs& w, int n, int total, bool elbo, const float* xb, const int* cb, int64_t bs) {
    w.ngroups = n; w.total_wgs = total; w.with_elbo = elbo; w.xbase = xb; w.cur_batch = cb; w.batch_stride = bs;
}
void set_head(WGradArgs3& w, int n, int total, bool elbo, const float* xb, const int* cb, int64_t bs) {
    W3Head& h = w.hd;
    h.ngroups = n; h.total_wgs = total; h.with_elbo = elbo; h.xbase = xb; h.cur_batch = cb; h.batch_stride = bs;
    h.gb1 = n > 1 ? w.g[1].wg_begin : total; h.gb2 = n > 2 ? w.g[2].wg_begin : total;
    h.nred = 0; h.red_cnt = nullptr;
}
int total_wgs(const WGradArgs& w) { return w.total_wgs; }
int total_wgs(const WGradArgs3& w) { return w.hd.total_wgs; }

// Weight-gradient arguments over `n` groups whose tiles start at block `base` of the
// launch (+ the ELBO workgroup when e != nullptr).  *vec: 16-byte panel loads are legal.
template <class WA>
int prep_wgrad(vaeb_ctx* c, const WGroup* groups, int n, const OptArgs& opt, const ElboArgs* e, const StepArgs& a,
               int base, WA& w, bool& vec, int tw, int* vmask = nullptr) {
    w = WA{};
    int begin = base;
    constexpr int kMaxG = (int)(sizeof(w.g) / sizeof(w.g[0]));
    if (n < 1 || n > kMaxG) return fail(VAEB_ERR_ARG, "internal: 1 to %d weight-gradient groups per launch", kMaxG);
    for (int gi = 0; gi < n; ++gi) {
        w.g[gi] = groups[gi];
        WGroup& G = w.g[gi];
        G.tiles_j = cdiv(G.N0 + G.N1, tw);
        G.wg_begin = begin;
        G.wg_end = begin + cdiv(G.rowsW + 1, kWT) * G.tiles_j;
        begin = G.wg_end;
    }
    set_head(w, n, begin, e != nullptr, a.xbase, c->ictl + 1, a.batch_stride);
    w.opt = opt;
    if (e) w.elbo = *e;
    w.P = c->P;
    w.dbg = a.dbg;
    // 16-byte panel loads need every panel row aligned with widths % 4 == 0 (the
    // activation buffers are hipMalloc'd; X rows are D floats apart)
    vec = true;
    if (vmask) *vmask = 0;
    auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    for (int gi = 0; gi < n; ++gi) {
        const WGroup& G = w.g[gi];
        // (and 16-byte theta / Adagrad-state accesses in the epilogue: arena offsets % 4 == 0)
        const bool gv = (G.ld_at % 4 == 0) && (G.rowsW % 4 == 0) && (G.at_is_x ? al(a.xbase) : al(G.at)) &&
                        (G.ld0 % 4 == 0) && (G.N0 % 4 == 0) && al(G.b0) && G.offW0 % 4 == 0 && G.offb0 % 4 == 0 &&
                        (G.N1 == 0 || ((G.ld1 % 4 == 0) && (G.N1 % 4 == 0) && al(G.b1) && G.offW1 % 4 == 0 &&
                                       G.offb1 % 4 == 0)) &&
                        al(c->theta2[0]) && al(c->theta2[1]) && al(c->acc) && al(c->grad);
        vec = vec && gv;
        if (vmask && gv) *vmask |= 1 << gi;
    }
    return 0;
}

// A standalone weight-gradient launch (256-thread blocks).  da3: group 0 (dW3) forms its
// dA3 panel from [dMu | dLv] in the workgroup (the folded latent backward).
int launch_wgrad(vaeb_ctx* c, hipStream_t s, const WGroup* groups, int n, const OptArgs& opt, const ElboArgs* e,
                 const StepArgs& a, const Da3Src* da3 = nullptr) {
    bool vec;
    if (da3) {
        if (n != 3) return fail(VAEB_ERR_ARG, "internal: the dA3-forming launch takes three groups");
        WGradArgs3 w;
        // 16-column tiles (32-wide: MNIST 46.3 vs 44.7 us, Frey 41.5 vs 38.4 in round 2;
        // -DVAEB_W3_TS=2 builds them for A/B)
        int vm = 0;   // 16-byte panel loads per group (Frey: dW3 yes, dW4 | dW5 and dW1 not)
        if (int rc = prep_wgrad(c, groups, n, opt, e, a, 0, w, vec, 16 * kW3TS, &vm)) return rc;
        w.da3 = *da3;
        const int nred = da3->red.nred;
        w.hd.nred = nred;
        w.hd.red_cnt = da3->red.cnt;
        const dim3 grid(w.hd.total_wgs + (e ? 1 : 0) + nred);
        auto go = [&](auto DF) {
            constexpr bool df = decltype(DF)::value;
            switch (vm) {
                case 7: hipLaunchKernelGGL((wgrad3_kernel<7, kW3TS, df>), grid, dim3(256), 0, s, w); break;
                case 1: hipLaunchKernelGGL((wgrad3_kernel<1, kW3TS, df>), grid, dim3(256), 0, s, w); break;
                case 3: hipLaunchKernelGGL((wgrad3_kernel<3, kW3TS, df>), grid, dim3(256), 0, s, w); break;
                case 5: hipLaunchKernelGGL((wgrad3_kernel<5, kW3TS, df>), grid, dim3(256), 0, s, w); break;
                default: hipLaunchKernelGGL((wgrad3_kernel<0, kW3TS, df>), grid, dim3(256), 0, s, w); break;
            }
        };
        // DEFER: reducers in this launch, or [dMu | dLv] handed in by the dhd launch
        if (nred > 0) go(std::true_type{});
        else go(std::false_type{});
    } else {
        WGradArgs w;
        if (int rc = prep_wgrad(c, groups, n, opt, e, a, 0, w, vec, kWTJ_W)) return rc;
        const dim3 grid(w.total_wgs + (e ? 1 : 0));
        if (vec) hipLaunchKernelGGL((wgrad_kernel<true, kWTJ_W / 16>), grid, dim3(256), 0, s, w);
        else hipLaunchKernelGGL((wgrad_kernel<false, kWTJ_W / 16>), grid, dim3(256), 0, s, w);
    }
    CHECK_LAUNCH();
    return 0;
}

WGroup make_group(vaeb_ctx* c, const float* at, int ld_at, int klim, int at_is_x, int rowsW, const float* b0, int ld0,
                  int N0, const float* b1, int ld1, int N1, int K, int pW0, int pb0, int pW1, int pb1) {
    WGroup G{};
    G.at = at; G.ld_at = ld_at; G.klim_at = klim; G.at_is_x = at_is_x; G.rowsW = rowsW;
    G.b0 = b0; G.ld0 = ld0; G.N0 = N0; G.b1 = b1; G.ld1 = ld1; G.N1 = N1; G.K = K;
    G.offW0 = c->off[pW0]; G.offb0 = c->off[pb0];
    G.offW1 = pW1 >= 0 ? c->off[pW1] : 0; G.offb1 = pb1 >= 0 ? c->off[pb1] : 0;
    return G;
}

// The dW2 (| dW6) weight-gradient group -- [hd | 1]^T [dA2 (| dA6)] -- as launch arguments
// whose tiles start at block `base`, with the optimizer `opt`.
int w2_args(vaeb_ctx* c, const StepArgs& a, const OptArgs& opt, int base, WGradArgs& w, bool& vec) {
    const bool gs = gaussian(c);
    const int bo = gs ? 6 : 5;
    WGroup g4 = make_group(c, c->hd, a.H, a.Me, 0, a.H, c->dA2, a.D, a.D, gs ? c->dA6 : nullptr, a.D, gs ? a.D : 0,
                           a.Me, 4, bo + 4, gs ? 5 : -1, gs ? bo + 5 : -1);
    return prep_wgrad(c, &g4, 1, opt, nullptr, a, base, w, vec, kWTJ_P5);
}

// Whether the step on `a` defers its dW2 into the next step's encoder launch (vaeb_ctx::dw2_defer).
// Only where the dhd launch hands its latent backward to the last launch (ho_dz 2): there the
// dW2 tiles bound the dhd launch.  With the counted atomic backward (small fan-in: Frey) the dhd
// launch is bound by that hand-off and hides dW2, while the encoder would pay for it: Frey
// 29.78 / 29.87 µs in-step vs 31.54 / 31.55 deferred.
bool dw2_deferrable(const vaeb_ctx* c) {
    const int est = c->c.estimator;
    StepArgs a{};
    a.H = c->c.H;   // (all enc_form reads of the training step's arguments)
    return c->dw2_defer && c->c.dtype == VAEB_DTYPE_F32 && c->comm == nullptr && est != VAEB_EST_FV && est != VAEB_EST_FVS &&
           fused_latent(c) && c->fold_bwd && enc_form(c, a, FvFold{}, nullptr, nullptr, nullptr);
}
bool dw2_deferred(const vaeb_ctx* c, const StepArgs& a) {
    const int hd = ho_dz(c);
    return dw2_deferrable(c) && hd == 2 && folded_latent(c, a);
}

// Run the pending step's dW2 (| dW6) + Adagrad now (their own launch; the device flag makes it
// a no-op when a later step's encoder already ran them): every host read or write of the
// parameters, the Adagrad state or the gradient, every evaluation, comes after it.
int w2_flush(vaeb_ctx* c) {
    if (!c || !c->w2_dirty) return 0;
    c->w2_dirty = false;
    const int par = c->par;   // the arena the next step reads: the pending dW2 writes W2' there
    StepArgs a = make_args(c, par, c->c.B, MODE_TRAIN, c->data, true);
    WGradArgs w;
    bool vec;
    if (int rc = w2_args(c, a, make_opt(c, par ^ 1, true, c->c.keep_grads != 0), 0, w, vec)) return rc;
    w.dbg = nullptr;
    if (vec) hipLaunchKernelGGL((w2_flush_kernel<true, kWTJ_P5 / 16>), dim3(w.total_wgs), dim3(512), 0, c->s, w, c->w2pend);
    else hipLaunchKernelGGL((w2_flush_kernel<false, kWTJ_P5 / 16>), dim3(w.total_wgs), dim3(512), 0, c->s, w, c->w2pend);
    CHECK_LAUNCH();
    HIP_TRY(hipMemsetAsync(c->w2pend, 0, sizeof(int), c->s));
    return 0;
}

// ------------------------------------------------------------------ DP gradient buckets
// Arena order W3 W4 W5 W1 W2 [W6] b3 b4 b5 b1 b2 [b6] | SGVB.  Bucket A = W2 [| W6] is final
// once the dW2 (| dW6) launch has run, early in the backward; bucket B = the rest plus the
// SGVB slot, final after the last weight-gradient launch.  Unprofiled steps fork bucket A's
// all-reduce and Adagrad onto s2, where they overlap the remaining backward launches; s
// then waits for bucket A's all-reduce (RCCL calls on one communicator stay serialised, in
// the same order on every rank), reduces bucket B itself, runs its Adagrad and waits for
// bucket A's Adagrad.  Only the fork sits on s2's queue: the critical path on s keeps its
// own queue, and both waits are normally satisfied by the time s reaches them.  Profiled
// steps run one all-reduce and one optimizer launch on s (per-kernel timing).
// The fork costs ~18 us per step on the fp32 engine's 58-us MNIST step at world 1 (hipGraph
// with a second branch; 78 vs 60 us) -- more than a 1.6-MB bucket's all-reduce can hide --
// so it is the bf16 engine's default only, where bucket A is 34 MB (config 5) and its
// Adagrad alone (37 us) pays for the fork already at world 1 (933 vs ~940 us).
// Sharded form (vaeb_ctx::dp_shard, world > 1): instead of all-reducing the
// whole bucket and running the replicated Adagrad over all of it on every rank, each rank
// reduce-scatters the bucket, updates ITS 1/W shard (prior + Adagrad; bf16: + shadow), and the
// shards of theta' are all-gathered: the same xGMI bytes as the all-reduce (a ring all-reduce
// is a reduce-scatter + all-gather), the optimizer stream per rank W times shorter, and every
// replica bitwise identical (theta' comes from one owner).  Shards are 64-element aligned; the
// remainder of each run (< 64 W elements, and the SGVB slot) is all-reduced and updated on
// every rank.  The arena is always partitioned into the same three runs -- B0 = [0, W2),
// A = [W2, b3) (W2 | W6), B1 = [b3, P) -- so an element's owner (and its Adagrad state, kept
// on the owner only) is the same whichever bucket form a step takes.
struct DpBucket {
    int nrun;
    int64_t lo[3], n[3];
    bool slot;   // + grad[P] (the SGVB), right after the run that ends at P (the last one)
};
DpBucket dp_bucket_a_runs(const vaeb_ctx* c) {
    const int bo = gaussian(c) ? 6 : 5;
    return DpBucket{1, {c->off[4], 0, 0}, {c->off[bo] - c->off[4], 0, 0}, false};
}
DpBucket dp_bucket_b_runs(const vaeb_ctx* c) {
    const int bo = gaussian(c) ? 6 : 5;
    return DpBucket{2, {0, c->off[bo], 0}, {c->off[4], c->P - c->off[bo], 0}, true};
}
DpBucket dp_bucket_all_runs(const vaeb_ctx* c) {
    const int bo = gaussian(c) ? 6 : 5;
    return DpBucket{3, {0, c->off[4], c->off[bo]}, {c->off[4], c->off[bo] - c->off[4], c->P - c->off[bo]}, true};
}
// elements per rank of a run of n (0: the run is all-reduced and updated everywhere)
int64_t dp_shard_len(const vaeb_ctx* c, int64_t n) { return c->dp_shard ? (n / c->world) & ~(int64_t)63 : 0; }
// what this rank's optimizer launch updates: each run's own shard and its replicated remainder
DpRange dp_opt_range(const vaeb_ctx* c, const DpBucket& bk) {
    DpRange r{};
    int k = 0;
    for (int j = 0; j < bk.nrun; ++j) {
        const int64_t S = dp_shard_len(c, bk.n[j]), tail = bk.n[j] - c->world * S;
        if (S) { r.lo[k] = bk.lo[j] + c->rank * S; r.n[k++] = S; }
        if (tail) { r.lo[k] = bk.lo[j] + c->world * S; r.n[k++] = tail; }
    }
    r.book = bk.slot ? 1 : 0;
    return r;
}
// the elements of the bucket other ranks updated (their shards): the bf16 shadow fix
DpRange dp_foreign_range(const vaeb_ctx* c, const DpBucket& bk) {
    DpRange r{};
    int k = 0;
    for (int j = 0; j < bk.nrun; ++j) {
        const int64_t S = dp_shard_len(c, bk.n[j]);
        if (!S) continue;
        if (c->rank > 0) { r.lo[k] = bk.lo[j]; r.n[k++] = c->rank * S; }
        if (c->rank < c->world - 1) { r.lo[k] = bk.lo[j] + (c->rank + 1) * S; r.n[k++] = (c->world - c->rank - 1) * S; }
    }
    return r;
}

// The fp32 engine's DP optimizer launch over range r (prior + Adagrad; r.book: also the SGVB
// bookkeeping): the step's dp_opt, and what vaeb_dp_rank_update runs for one emulated rank.
int dp_opt_launch(vaeb_ctx* c, hipStream_t st, const OptArgs& o, const DpRange& r, const ElboArgs& e) {
    int64_t n = 0;
    for (int k = 0; k < kDpRuns; ++k) n += r.n[k];
    // (sharded: a 1/W share of the arena; the grid scales down with it)
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(r.book ? 512 : 256, cdiv(n, 256 * 8)));
    hipLaunchKernelGGL(adagrad_kernel, dim3(nb), dim3(256), 0, st, o, c->P, r, e);
    CHECK_LAUNCH();
    return 0;
}

int nccl_ok(ncclResult_t r, const char* what) {
    return r == ncclSuccess ? 0 : fail(VAEB_ERR_COMM, "%s: %s", what, ncclGetErrorString(r));
}
int nccl_sum(vaeb_ctx* c, float* p, int64_t n, hipStream_t st) {
    return nccl_ok(ncclAllReduce(p, p, (size_t)n, ncclFloat, ncclSum, c->comm, st), "ncclAllReduce");
}

// One bucket on stream st: the reduction (reduce-scatter of each run's shards + all-reduce of
// the remainders and the slot, one RCCL group), this rank's optimizer launch, then (sharded)
// the all-gather of theta' shards and fix(st, foreign range) for the bf16 shadow.  comm_done
// (if any) is recorded after the bucket's last collective: another stream's collectives wait
// for it (RCCL calls on one communicator stay serialised, in the same order on every rank).
template <class Opt, class Fix>
int dp_reduce_update(vaeb_ctx* c, hipStream_t st, const DpBucket& bk, float* theta_out, Opt opt, Fix fix,
                     hipEvent_t comm_done, Prof* pr = nullptr, int opt_mark = -1) {
    const int W = c->world, rk = c->rank;
    bool sharded = false;
    if (pr) pr->mark(8);
    for (int rep = 0; rep < (pr ? pr->reps : 1); ++rep) {
        if (int rc = nccl_ok(ncclGroupStart(), "ncclGroupStart")) return rc;
        int rc = 0;
        for (int j = 0; j < bk.nrun && !rc; ++j) {
            const int64_t S = dp_shard_len(c, bk.n[j]);
            const int64_t tail = bk.n[j] - W * S + ((bk.slot && j == bk.nrun - 1) ? 1 : 0);
            float* g = c->grad + bk.lo[j];
            if (S) {
                sharded = true;
                rc = nccl_ok(ncclReduceScatter(g, g + rk * S, (size_t)S, ncclFloat, ncclSum, c->comm, st),
                             "ncclReduceScatter");
            }
            if (!rc && tail) rc = nccl_sum(c, g + W * S, tail, st);
        }
        const int re = nccl_ok(ncclGroupEnd(), "ncclGroupEnd");
        if (rc) return rc;
        if (re) return re;
    }
    if (comm_done && !sharded) HIP_TRY(hipEventRecord(comm_done, st));
    if (pr) pr->mark(opt_mark);
    for (int rep = 0; rep < (pr ? pr->reps : 1); ++rep)
        if (int rc = opt(st, dp_opt_range(c, bk))) return rc;
    if (!sharded) return 0;
    if (int rc = nccl_ok(ncclGroupStart(), "ncclGroupStart")) return rc;
    int rc = 0;
    for (int j = 0; j < bk.nrun && !rc; ++j) {
        const int64_t S = dp_shard_len(c, bk.n[j]);
        float* t = theta_out + bk.lo[j];
        if (S) rc = nccl_ok(ncclAllGather(t + rk * S, t, (size_t)S, ncclFloat, c->comm, st), "ncclAllGather");
    }
    const int re = nccl_ok(ncclGroupEnd(), "ncclGroupEnd");
    if (rc) return rc;
    if (re) return re;
    if (comm_done) HIP_TRY(hipEventRecord(comm_done, st));
    return fix(st, dp_foreign_range(c, bk));
}

// Sharded Adagrad keeps each element's accumulator on its owner only: gather the shards before
// the host reads the state (vaeb_get_adagrad_state, vaeb_checkpoint_save; every rank calls it).
int dp_gather_acc(vaeb_ctx* c) {
    if (!c->comm || !c->dp_shard) return 0;
    const DpBucket bk = dp_bucket_all_runs(c);
    if (int rc = nccl_ok(ncclGroupStart(), "ncclGroupStart")) return rc;
    int rc = 0;
    for (int j = 0; j < bk.nrun && !rc; ++j) {
        const int64_t S = dp_shard_len(c, bk.n[j]);
        float* t = c->acc + bk.lo[j];
        if (S) rc = nccl_ok(ncclAllGather(t + c->rank * S, t, (size_t)S, ncclFloat, c->comm, c->s), "ncclAllGather");
    }
    const int re = nccl_ok(ncclGroupEnd(), "ncclGroupEnd");
    if (rc) return rc;
    if (re) return re;
    HIP_TRY(hipStreamSynchronize(c->s));
    return 0;
}

// after the dW2 (| dW6) launch: opt(stream, range) enqueues the optimizer over a range,
// fix(stream, range) the bf16 shadow of other ranks' shards (fp32: nothing)
template <class Opt, class Fix>
int dp_bucket_a(vaeb_ctx* c, const Prof& pr, float* theta_out, Opt opt, Fix fix) {
    if (pr.on || !c->dp_overlap) return 0;
    HIP_TRY(hipEventRecord(c->dp_ev[0], c->s));
    HIP_TRY(hipStreamWaitEvent(c->s2, c->dp_ev[0], 0));
    if (int rc = dp_reduce_update(c, c->s2, dp_bucket_a_runs(c), theta_out, opt, fix, c->dp_ev[1])) return rc;
    HIP_TRY(hipEventRecord(c->dp_ev[2], c->s2));
    return 0;
}

// after the last weight-gradient launch (the SGVB slot written)
template <class Opt, class Fix>
int dp_bucket_b(vaeb_ctx* c, Prof& pr, int opt_mark, float* theta_out, Opt opt, Fix fix) {
    if (pr.on || !c->dp_overlap)
        return dp_reduce_update(c, c->s, dp_bucket_all_runs(c), theta_out, opt, fix, nullptr, pr.on ? &pr : nullptr,
                                opt_mark);
    HIP_TRY(hipStreamWaitEvent(c->s, c->dp_ev[1], 0));
    if (int rc = dp_reduce_update(c, c->s, dp_bucket_b_runs(c), theta_out, opt, fix, nullptr)) return rc;
    HIP_TRY(hipStreamWaitEvent(c->s, c->dp_ev[2], 0));
    return 0;
}

// ------------------------------------------------------------------ the 16-bit engine
// One host engine (engine_bf16.inc) over two device instantiations (h16_engines.hpp): bf16
// (VAEB_DTYPE_BF16) and fp16 (VAEB_DTYPE_F16) operands, fp32 accumulation, fp32 masters.
using bf::bf16_t;
bool is_bf16(const vaeb_ctx* c) { return c->c.dtype == VAEB_DTYPE_BF16 || c->c.dtype == VAEB_DTYPE_F16; }   // the 16-bit engine
bool is_f16(const vaeb_ctx* c) { return c->c.dtype == VAEB_DTYPE_F16; }
// A/B (round 3): 256 x 256 tiles on the 8-phase BK = 64 main loop (gemm8_kernel) instead of
// gemm_body's BK = 32 ring, per operand-layout pair: bit (2 LA + LB) of VAEB_BF_GEMM8 (set at
// context creation) -- 1: KC x KC (dhd), 2: KC x KO (enc), 8: KO x KO (dW2, dW3).
int g_gemm8 = 0;
template <int LA, int LB> bool use8() { return (g_gemm8 >> (2 * LA + LB)) & 1; }
// A forward pass of the 16-bit engine for `Mb` rows starting at x (device, 16-bit) with the
// parameters of arena par.  train: store dA / bias partials for the backward.  yout: decoder means.
struct BfFwd {
    int Mb, mode; bool train;
    const bf16_t* x; h16c::BatchRef xb;
    const uint32_t* xbits = nullptr;   // x as bits (binary datasets; the training step's rows), or null
    int64_t row_base_mul, row_base_add;
    const float* eps_in; int64_t eps_in_ld; uint32_t domain;
    float* yout;
};
namespace eng_bf {
namespace bf = ::vaeb::bf;
constexpr bool kF16 = false;
#include "engine_bf16.inc"
}  // namespace eng_bf
namespace eng_hf {
namespace bf = ::vaeb::hf;
constexpr bool kF16 = true;
#include "engine_bf16.inc"
}  // namespace eng_hf
#define H16_CALL(fn, ...) (is_f16(c) ? eng_hf::fn(__VA_ARGS__) : eng_bf::fn(__VA_ARGS__))
int bf_train_step(vaeb_ctx* c, int par, bool prof, int direct) { return H16_CALL(bf_train_step, c, par, prof, direct); }
int bf_alloc(vaeb_ctx* c) { return H16_CALL(bf_alloc, c); }
void bf_free(vaeb_ctx* c) { eng_bf::bf_free(c); }   // (type-independent: frees the state's buffers)
int bf_make_shadow(vaeb_ctx* c, int par) { return H16_CALL(bf_make_shadow, c, par); }
int bf_upload_rows(vaeb_ctx* c, const float* x, int64_t n, bf16_t* dst) { return H16_CALL(bf_upload_rows, c, x, n, dst); }
int bf_forward(vaeb_ctx* c, int par, const BfFwd& f, Prof& pr) { return H16_CALL(bf_forward, c, par, f, pr); }
int bf_eval_chunk(vaeb_ctx* c, const float* x, int rows, int64_t r0, int mode, float* out_y) {
    return H16_CALL(bf_eval_chunk, c, x, rows, r0, mode, out_y);
}
int bf_eval_chunk_dev(vaeb_ctx* c, const bf16_t* x, int rows, int64_t r0, int mode, float* out_y) {
    return H16_CALL(bf_eval_chunk_dev, c, x, rows, r0, mode, out_y);
}
int h16_dp_opt(vaeb_ctx* c, int par, const DpRange& own) { return H16_CALL(h16_dp_opt, c, par, own); }
int h16_dp_fix(vaeb_ctx* c, int par, const DpRange& fr) { return H16_CALL(h16_dp_fix, c, par, fr); }

// One training step reading parameter arena `par` and writing arena par ^ 1.
// One stream: P1 -> P23 -> P4 -> [P5 | dW2 (| dW6)] -> [P67 | dW1] -> [dW3 | dW45 + ELBO]
// (bracketed groups share one grid, see hfuse.hpp); DP adds all-reduce -> Adagrad.
// `prof` brackets every launch with timing events.
// fresh: first step of an enqueued sequence (VAEB_EST_FVS in Philox mode draws the weight
// sample here; later steps of the sequence read the one their predecessor's update wrote).
// direct >= 0: the step's minibatch index given by the host (vaeb_update's single eager
// step): the rows are addressed from the launch arguments, no order upload, no cursor.
int enqueue_train_step(vaeb_ctx* c, int par, bool prof, bool fresh = true, int direct = -1) {
    if (is_bf16(c)) return bf_train_step(c, par, prof, direct);
    Prof pr{c, prof};
    if (prof) pr.reps = c->prof_reps;
    const vaeb_config& g = c->c;
    hipStream_t s = c->s;
    // VAEB_EST_FVS: the step reads the weight sample theta~ written into the spare arena
    // par ^ 1 (the loaded theta in arena par is never updated, as on the literal path)
    const bool fvs = g.estimator == VAEB_EST_FVS;
    const float* zin = (fvs && c->eps_mode == VAEB_EPS_HOST) ? c->fvzeta : nullptr;
    if (fvs && (fresh || zin)) {
        pr.mark(37);
        REP(pr) hipLaunchKernelGGL(fvs_sample_kernel, dim3(kFvParts), dim3(256), 0, s, c->fvmu, c->fvsg,
                                   c->theta2[par ^ 1], c->P, c->seed, c->step, zin);
        CHECK_LAUNCH();
    }
    if (fvs) par ^= 1;
    StepArgs a = make_args(c, par, g.B, g.estimator == VAEB_EST_FV ? MODE_EVAL : MODE_TRAIN, c->data, true);
    if (direct >= 0) {
        const int64_t row0 = (int64_t)direct * g.B_global + g.row_offset;
        a.order = nullptr;
        a.xbase = c->data + row0 * g.D;
        a.batch_stride = 0;
        a.row_base_mul = 0;
        a.row_base_add = row0;
    }
    // literal FV: the (mu, sigma) update needs none of the step's data; with the folded
    // latent block it rides enc_latent_kernel's extra grid rows (~256 blocks), else it is
    // fv_kernel's launch
    const bool fv_fold = g.estimator == VAEB_EST_FV && folded_latent(c, a);
    int n_fv = kFvParts;
    FvFold fvf{};
    if (fv_fold) {
        fvf = FvFold{c->fvmu, c->fvsg, c->fvam, c->fvas, c->fv_part, c->P, g.lr, g.adagrad_eps, cdiv(256, a.Mbp / 16)};
        n_fv = fvf.rows * (a.Mbp / 16);
        if (n_fv > kFvParts) return fail(VAEB_ERR_ARG, "internal: %d FV partials > %d", n_fv, kFvParts);
    }
    // the deferred dW2: the PREVIOUS step's dW2 (| dW6) rides this step's encoder launch --
    // theta from the other arena, theta' into this step's (make_opt(par ^ 1)); this step's own
    // dW2 is left pending for the next step (or a flush)
    const bool w2d = dw2_deferred(c, a);
    W2Launch w2{};
    if (w2d) {
        if (int rc = w2_args(c, a, make_opt(c, par ^ 1, true, g.keep_grads != 0), 0, w2.w, w2.vec)) return rc;
        // (timeline build: the dW2 tiles stamp at logical ids 256 + tile of the encoder launch)
        w2.w.dbg = c->dbg ? c->dbg + (size_t)c->dbg_slot * kDbgWG * 8 + 256 * 8 : nullptr;
        w2.pend = c->w2pend;
    }
    if (int rc = enqueue_forward(c, a, pr, fvf, w2d ? &w2 : nullptr)) return rc;
    ElboArgs e = base_elbo(c, a);
    e.elbo_out = c->elbo_out; e.epoch = c->epoch; e.cursor = direct >= 0 ? nullptr : c->ictl; e.step = c->step;

    if (g.estimator == VAEB_EST_FV) {
        if (!fv_fold) {
            pr.mark(10);
            REP(pr) hipLaunchKernelGGL(fv_kernel, dim3(kFvParts), dim3(256), 0, s, c->fvmu, c->fvsg, c->fvam,
                                       c->fvas, c->P, g.lr, g.adagrad_eps, 1, c->fv_part);
            CHECK_LAUNCH();
        }
        pr.mark(11);
        e.fv_part = c->fv_part; e.n_fv = n_fv;
        e.data_mul = (double)g.B;
        hipLaunchKernelGGL(elbo_kernel, dim3(1), dim3(256), 0, s, e);
        CHECK_LAUNCH();
        pr.mark(-1);
        c->prof_n = pr.k;
        return 0;
    }
    const bool dp = c->comm != nullptr;  // any communicator (also world 1) takes the all-reduce path
    // FVS: the weight-gradient launches only store the data gradient at theta~
    const OptArgs opt = make_opt(c, par, !dp && !fvs, dp || fvs || g.keep_grads != 0);
    const int bo = gaussian(c) ? 6 : 5;
    const bool gs = gaussian(c);
    const OptArgs dopt = make_opt(c, par, true, false);
    auto dp_opt = [&](hipStream_t st, const DpRange& r) -> int { return dp_opt_launch(c, st, dopt, r, e); };

    // folded latent backward (Z <= 32, latent_bwd.hpp): the dhd launch also finishes dZ and
    // [dMu | dLv]; dA3 is formed inside the dW3 workgroups of the last launch (with dW1)
    const bool fold = fused_latent(c) && c->fold_bwd;
    // P5 + dW2 (| dW6) = [hd|1]^T [dA2 (| dA6)] in one grid: both need only P4's outputs
    a.dbg = next_dbg(c);
    if (fold) {
        WGroup g4 = make_group(c, c->hd, a.H, a.Me, 0, a.H, c->dA2, a.D, a.D, gs ? c->dA6 : nullptr, a.D, gs ? a.D : 0,
                               a.Me, 4, bo + 4, gs ? 5 : -1, gs ? bo + 5 : -1);
        const PDhdT<true> p5{a, a.Me, a.H, gs ? ((a.D + 3) & ~3) + a.D : a.D};
        const PDhdT<false> p5s{a, a.Me, a.H, p5.K};
        const int gx = cdiv(p5.M, 16), ntile = gx * cdiv(p5.N, 16);
        WGradArgs w;
        bool vec;
        if (int rc = prep_wgrad(c, &g4, 1, opt, nullptr, a, ntile, w, vec, kWTJ_P5)) return rc;
        // the dhd loaders' 16-byte form needs D % 4 == 0 and aligned dA2 / W2 too
        vec = vec && dhd_vec(a);
        DhdAux pend{nullptr};
        if (w2d) {   // no dW2 tiles here: the next step's encoder launch (or a flush) runs them
            w.total_wgs = ntile;
            pend.pend = c->w2pend;
        }
        const dim3 grid(w.total_wgs);
        const bool deep = cdiv(cdiv(p5.K, 16), 8) > 4;
        pr.mark(w2d ? 43 : 39);
        REP(pr) {
            switch (ho_dz(c)) {
                case 1: launch_dhd_dz<kWTJ_P5 / 16, 1>(s, grid, p5, p5s, w, ntile, gx, vec, deep, pend); break;
                case 2: launch_dhd_dz<kWTJ_P5 / 16, 2>(s, grid, p5, p5s, w, ntile, gx, vec, deep, pend); break;
                default: launch_dhd_dz<kWTJ_P5 / 16, 0>(s, grid, p5, p5s, w, ntile, gx, vec, deep, pend); break;
            }
        }
        CHECK_LAUNCH();
        if (w2d) c->w2_dirty = true;
    } else {
        WGroup g4 = make_group(c, c->hd, a.H, a.Me, 0, a.H, c->dA2, a.D, a.D, gs ? c->dA6 : nullptr, a.D, gs ? a.D : 0,
                               a.Me, 4, bo + 4, gs ? 5 : -1, gs ? bo + 5 : -1);
        const PDhdT<true> p5{a, a.Me, a.H, gs ? ((a.D + 3) & ~3) + a.D : a.D};
        const PDhdT<false> p5s{a, a.Me, a.H, p5.K};
        const int gx = cdiv(p5.M, 16), ntile = gx * cdiv(p5.N, 16);
        WGradArgs w;
        bool vec;
        if (int rc = prep_wgrad(c, &g4, 1, opt, nullptr, a, ntile, w, vec, kWTJ_P5)) return rc;
        vec = vec && dhd_vec(a);
        const dim3 grid(w.total_wgs);
        pr.mark(4);
        REP(pr) if (cdiv(cdiv(p5.K, 16), 8) <= 4) {
            if (vec) hipLaunchKernelGGL((tile_wgrad_kernel<1, 1, 8, 1, 4, PDhdT<true>, true, kWTJ_P5 / 16>), grid, dim3(512), 0, s, p5, w, ntile, gx);
            else hipLaunchKernelGGL((tile_wgrad_kernel<1, 1, 8, 1, 4, PDhdT<false>, false, kWTJ_P5 / 16>), grid, dim3(512), 0, s, p5s, w, ntile, gx);
        } else {
            if (vec) hipLaunchKernelGGL((tile_wgrad_kernel<1, 1, 8, 1, 8, PDhdT<true>, true, kWTJ_P5 / 16>), grid, dim3(512), 0, s, p5, w, ntile, gx);
            else hipLaunchKernelGGL((tile_wgrad_kernel<1, 1, 8, 1, 8, PDhdT<false>, false, kWTJ_P5 / 16>), grid, dim3(512), 0, s, p5s, w, ntile, gx);
        }
        CHECK_LAUNCH();
    }
    auto no_fix = [](hipStream_t, const DpRange&) -> int { return 0; };
    if (dp) if (int rc = dp_bucket_a(c, pr, dopt.theta_out, dp_opt, no_fix)) return rc;
    // P67 (+ dW1 = [z|1]^T dA1 on the fused path): both need only P5's output
    if (!fold) {
        a.dbg = next_dbg(c);
        WGroup g3 = make_group(c, c->z, a.Z, a.Me, 0, a.Z, c->dA1, a.H, a.H, nullptr, 0, 0, a.Me, 3, bo + 3, -1, -1);
        if (fused_latent(c)) {
            const int nrow = a.Mbp / 16 * std::max(1, std::min(kDzSplit, cdiv(a.H, 16)));
            WGradArgs w;
            bool vec;
            if (int rc = prep_wgrad(c, &g3, 1, opt, nullptr, a, nrow, w, vec, kWTJ_P67)) return rc;
            const dim3 grid(w.total_wgs);
            pr.mark(13);
            REP(pr) if (a.Z <= 16) {
                if (vec) hipLaunchKernelGGL((dz_dh_wgrad_kernel<1, true, kWTJ_P67 / 16>), grid, dim3(512), 0, s, a, w, nrow);
                else hipLaunchKernelGGL((dz_dh_wgrad_kernel<1, false, kWTJ_P67 / 16>), grid, dim3(512), 0, s, a, w, nrow);
            } else {
                if (vec) hipLaunchKernelGGL((dz_dh_wgrad_kernel<2, true, kWTJ_P67 / 16>), grid, dim3(512), 0, s, a, w, nrow);
                else hipLaunchKernelGGL((dz_dh_wgrad_kernel<2, false, kWTJ_P67 / 16>), grid, dim3(512), 0, s, a, w, nrow);
            }
            CHECK_LAUNCH();
        } else {
            pr.mark(15);
            REP(pr) if (int rc = launch_wgrad(c, s, &g3, 1, opt, nullptr, a)) return rc;
            a.dbg = next_dbg(c);
            pr.mark(5);
            REP(pr) launch_tile<1, 1, 4, 1, 8>(s, PDz{a, a.Me, a.Z, a.H});
            CHECK_LAUNCH();
            a.dbg = next_dbg(c);
            pr.mark(6);
            REP(pr) launch_tile<1, 4, 1, 1, 8>(s, PDh{a, a.Mbp, a.H, 2 * a.Z});
            CHECK_LAUNCH();
        }
    }
    // dW3 = [X|1]^T dA3 and dW4|dW5 = [h|1]^T [dMu|dLv] (+ dW1 = [z|1]^T dA1 when the latent
    // backward is folded: dA3 is then formed in the dW3 workgroups), plus the ELBO workgroup
    {
        WGroup g12[3] = {
            make_group(c, nullptr, a.D, a.Mb, 1, a.D, c->dA3, a.H, a.H, nullptr, 0, 0, a.Mbp, 0, bo + 0, -1, -1),
            make_group(c, c->h, a.H, a.Mbp, 0, a.H, c->dMuLv, 2 * a.Z, a.Z, c->dMuLv + a.Z, 2 * a.Z, a.Z, a.Mbp, 1,
                       bo + 1, 2, bo + 2),
            make_group(c, c->z, a.Z, a.Me, 0, a.Z, c->dA1, a.H, a.H, nullptr, 0, 0, a.Me, 3, bo + 3, -1, -1)};
        ElboArgs e1 = e;
        if (dp || fvs) { e1.dp_slot = c->grad + c->P; e1.elbo_out = nullptr; e1.cursor = nullptr; e1.step = nullptr; }
        a.dbg = next_dbg(c);
        if (fold) {
            Da3Src d3{c->dMuLv, a.W4, a.W5, c->h, c->dA3, a.Z, a.H, a.Mb, a.Mbp, LatRed{}};
            if (ho_dz(c) == 2) {
                // the deferred latent backward: ceil(Z / 8) column groups per 16-row block
                LatRed& r = d3.red;
                r.slab = c->slab_dz; r.mu = c->mu; r.lv = c->lv; r.eps = c->eps; r.z = c->z;
                r.dZ = c->dZ; r.dml = c->dMuLv; r.cnt = c->cnt_dz; r.guard = c->blk + kBlkFxErr;
                // (Z % 4 == 0: groups of a multiple of 4 latents, so VAEB_LAT_ST4 reducers can
                // publish whole 16-byte runs; MNIST-20: 8, 8, 4)
                r.ngrp = cdiv(a.Z, 8); r.zg = cdiv(a.Z, r.ngrp);
                if (a.Z % 4 == 0) { r.zg = (r.zg + 3) & ~3; r.ngrp = cdiv(a.Z, r.zg); }
                r.nred = (a.Mbp / 16) * r.ngrp;
                r.nctH = cdiv(a.H, 16); r.L = a.L; r.est = a.est; r.Mb = a.Mb; r.Mbp = a.Mbp; r.Z = a.Z; r.sc = a.sc;
            }
            pr.mark(40);
            REP(pr) if (int rc = launch_wgrad(c, s, g12, 3, opt, &e1, a, &d3)) return rc;
        } else {
            pr.mark(7);
            REP(pr) if (int rc = launch_wgrad(c, s, g12, 2, opt, &e1, a)) return rc;
        }
    }
    if (fvs) {   // Adagrad on (mu_theta, sigma_theta), then the step's SGVB / B and cursor++
        pr.mark(38);
        REP(pr) hipLaunchKernelGGL(fvs_update_kernel, dim3(kFvParts), dim3(256), 0, s, c->fvmu, c->fvsg, c->fvam,
                                   c->fvas, (const float*)c->grad, c->P, (float)g.B, g.lr, g.adagrad_eps, c->seed,
                                   (const int64_t*)c->step, zin, c->fv_part, zin ? nullptr : c->theta2[par]);
        CHECK_LAUNCH();
        pr.mark(11);
        e.fv_part = c->fv_part; e.n_fv = kFvParts;
        e.data_mul = (double)g.B;
        e.est = VAEB_EST_FV;   // SGVB = B (sum log p + sum KL) + thetaPrior (VAEB.py:364)
        hipLaunchKernelGGL(elbo_kernel, dim3(1), dim3(256), 0, s, e);
        CHECK_LAUNCH();
    }
    if (dp) if (int rc = dp_bucket_b(c, pr, 9, dopt.theta_out, dp_opt, no_fix)) return rc;
    pr.mark(-1);
    c->prof_n = pr.k;
    return 0;
}

bool flips(const vaeb_ctx* c) { return c->c.estimator != VAEB_EST_FV && c->c.estimator != VAEB_EST_FVS; }

void free_graphs(vaeb_ctx* c) {
    for (auto& fam : c->gN)
        for (auto& gn : fam) {
            if (gn) hipGraphExecDestroy(gn);
            gn = nullptr;
        }
    c->w2_graph = false;
}

// Capture nsteps consecutive steps starting from parameter arena `par`.
int capture(vaeb_ctx* c, int nsteps, int par, hipGraphExec_t* out) {
    hipGraph_t gr = nullptr;
    HIP_TRY(hipStreamBeginCapture(c->s, hipStreamCaptureModeThreadLocal));
    int rc = 0;
    // a captured deferred-dW2 step sets w2_dirty as it is recorded; what the host must know is
    // that every REPLAY leaves a dW2 pending: w2_graph, applied by run_steps
    const bool dirty0 = c->w2_dirty;
    c->w2_dirty = false;
    for (int i = 0; i < nsteps && rc == 0; ++i) {
        rc = enqueue_train_step(c, par, false, i == 0);
        if (flips(c)) par ^= 1;
    }
    if (c->w2_dirty) c->w2_graph = true;
    c->w2_dirty = dirty0;
    hipError_t e = hipStreamEndCapture(c->s, &gr);
    if (rc) { if (gr) hipGraphDestroy(gr); return rc; }
    if (e != hipSuccess) return fail(VAEB_ERR_HIP, "hipStreamEndCapture: %s", hipGetErrorString(e));
    e = hipGraphInstantiate(out, gr, nullptr, nullptr, 0);
    hipGraphDestroy(gr);
    if (e != hipSuccess) return fail(VAEB_ERR_HIP, "hipGraphInstantiate: %s", hipGetErrorString(e));
    // upload now, with the capture: a graph's first launch otherwise pays it inside the call
    // that replays it (the driver's 20-step form replays a graph the warm-up never launched)
    if (hipGraphUpload(*out, c->s) != hipSuccess) (void)hipGetLastError();
    return 0;
}

int step_eager(vaeb_ctx* c, int direct = -1) {
    if (int rc = enqueue_train_step(c, c->par, false, true, direct)) return rc;
    if (flips(c)) c->par ^= 1;
    return 0;
}

// Enqueue n steps (graph replay when enabled, else eager launches).  Graphs: gN[p][m] is m
// steps from arena p (m = 1 .. 32; p = 1 only for the estimators that flip arenas), both
// families captured at the first call (a capture inside a later, timed call would cost more
// than the launches it saves).  A call replays as n / 32 launches of gN[par][32] + ONE launch
// of gN[par][n % 32] from whichever arena it starts: a graph-to-graph boundary leaves the GPU
// idle for ~8 us (kernel trace, profiles/r6/call_timeline.txt), so a 20-step call is one
// graph, not 16 + 4, and the 19 steps after update_many's eager first step are one graph,
// not [one step back to arena 0] + the arena-0 graph (rounds 3-5).
int run_steps(vaeb_ctx* c, int n) {
    if (c->c.use_graph && !c->graph_failed) {
        if (!c->gN[0][1]) {
            int rc = 0;
            for (int p = 0; p < (flips(c) ? 2 : 1); ++p)
                for (int m = 1; m <= kGraphSteps && rc == 0; ++m) rc = capture(c, m, p, &c->gN[p][m]);
            if (rc) {
                // never silent: the reason is kept for vaeb_graph_status.  With a
                // communicator of more than one rank the call fails instead of degrading:
                // single steps (vaeb_update, the first step of a call) are eager at any
                // world size and tested against replay (test_gpu_api.py), but a failed
                // capture there means RCCL could not be captured, and a multi-rank run would
                // then time a launch-bound form nobody asked for
                c->graph_failed = true;
                c->graph_err = g_err;
                free_graphs(c);
                (void)hipGetLastError();
                if (c->comm && c->world > 1)
                    return fail(VAEB_ERR_HIP, "graph capture of the data-parallel step failed at world %d: %s",
                                c->world, c->graph_err.c_str());
            }
        }
        if (!c->graph_failed) {
            // FV / FVS never flip the arena: c->par stays 0 and only family 0 exists
            for (int i = 0; i < n;) {
                const int m = std::min(kGraphSteps, n - i), p = flips(c) ? c->par : 0;
                HIP_TRY(hipGraphLaunch(c->gN[p][m], c->s));
                if (flips(c)) c->par = p ^ (m & 1);
                i += m;
            }
            if (n > 0 && c->w2_graph) c->w2_dirty = true;   // the last replayed step left its dW2 pending
            return 0;
        }
    }
    for (int i = 0; i < n; ++i)
        if (int rc = step_eager(c)) return rc;
    return 0;
}

// The order upload update_many held back for its eager first step (vaeb_ctx::order_pending):
// launched right after that step's first kernel, or after the step where no launch site
// takes it.  The eager step addresses its rows from its launch arguments and reads neither the
// order nor the cursor, so the upload may run between its launches.
int order_hook(vaeb_ctx* c) {
    if (!c->order_pending) return 0;
    c->order_pending = false;
    hipLaunchKernelGGL(set_order_kernel, dim3(1), dim3(256), 0, c->s, c->ictl, c->order_pend);
    CHECK_LAUNCH();
    return 0;
}

// Upload a batch order (cursor reset to 0).  Up to kArgOrder entries travel as a kernel
// argument of set_order_kernel (a kernel on the step stream starts sooner than a host ->
// device copy: the fixed cost of a short update_many call), longer ones through the
// pinned staging buffer in one contiguous copy of [cursor, cur_batch, next, order...].
int upload_order(vaeb_ctx* c, const int32_t* idx, int n) {
    if (n <= kArgOrder) {
        OrderArg u;
        u.n = n;
        memcpy(u.v, idx, sizeof(int) * (size_t)n);
        hipLaunchKernelGGL(set_order_kernel, dim3(1), dim3(256), 0, c->s, c->ictl, u);
        CHECK_LAUNCH();
        return 0;
    }
    HIP_TRY(hipEventSynchronize(c->ctl_ev));
    c->h_ctl[0] = 0;
    c->h_ctl[1] = 0;
    c->h_ctl[kCtlNext] = n > 0 ? idx[0] : 0;
    memcpy(c->h_ctl + kCtlOrder, idx, sizeof(int) * (size_t)n);
    HIP_TRY(hipMemcpyAsync(c->ictl, c->h_ctl, sizeof(int) * (size_t)(n + kCtlOrder), hipMemcpyHostToDevice, c->s));
    HIP_TRY(hipEventRecord(c->ctl_ev, c->s));
    return 0;
}

int check_batches(vaeb_ctx* c, const int32_t* idx, int n) {
    if (!c->data) return fail(VAEB_ERR_STATE, "vaeb_set_data has not been called");
    const int64_t nb = c->nrows / c->c.B_global;
    for (int i = 0; i < n; ++i)
        if (idx[i] < 0 || idx[i] >= nb)
            return fail(VAEB_ERR_ARG, "batch index %d out of range [0, %lld)", idx[i], (long long)nb);
    return 0;
}


}  // namespace

// =========================================================================== C ABI
extern "C" {

const char* vaeb_last_error(void) { return g_err.c_str(); }

int vaeb_version(int32_t* major, int32_t* minor) {
    if (major) *major = 0;
    if (minor) *minor = 1;
    return 0;
}

int vaeb_create(const vaeb_config* cfg, vaeb_ctx** out) {
    if (!cfg || !out) return fail(VAEB_ERR_ARG, "null argument");
    const vaeb_config& g = *cfg;
    if (g.D <= 0 || g.H <= 0 || g.Z <= 0 || g.B <= 0 || g.L <= 0)
        return fail(VAEB_ERR_ARG, "dimensions must be positive (D=%d H=%d Z=%d B=%d L=%d)", g.D, g.H, g.Z, g.B, g.L);
    if (g.decoder < 0 || g.decoder > 1 || g.estimator < 0 || g.estimator > 3 || g.objective < 0 || g.objective > 1)
        return fail(VAEB_ERR_ARG, "bad decoder/estimator/objective enum");
    const bool fvx = g.estimator == VAEB_EST_FV || g.estimator == VAEB_EST_FVS;
    if (fvx && g.L != 1)
        return fail(VAEB_ERR_ARG, "the full-variational estimators support L == 1 only (VAEB.py:361)");
    if (g.dtype != VAEB_DTYPE_F32 && g.dtype != VAEB_DTYPE_BF16 && g.dtype != VAEB_DTYPE_F16)
        return fail(VAEB_ERR_ARG, "bad dtype %d", g.dtype);
    if (g.dtype == VAEB_DTYPE_BF16 || g.dtype == VAEB_DTYPE_F16) {
        if (g.D % 8 || g.H % 8 || g.Z % 8)
            return fail(VAEB_ERR_ARG, "bf16 engine: D, H, Z must be multiples of 8 (got %d, %d, %d)", g.D, g.H, g.Z);
        if (g.decoder == VAEB_DEC_GAUSSIAN && g.D % 32)
            return fail(VAEB_ERR_ARG, "bf16 engine: the Gaussian decoder needs D %% 32 == 0 (got %d)", g.D);
        if (fvx) return fail(VAEB_ERR_ARG, "bf16 engine: the FV estimators run on the fp32 path");
        if (g.estimator == VAEB_EST_LA && g.L > 8) return fail(VAEB_ERR_ARG, "bf16 engine: LA supports L <= 8");
    }
    auto* c = new vaeb_ctx();
    c->c = g;
    if (c->c.B_global <= 0) c->c.B_global = g.B;
    if (c->c.adagrad_eps <= 0.f) c->c.adagrad_eps = 1e-6f;
    if (c->c.max_eval_rows <= 0) c->c.max_eval_rows = 10000;
    hipError_t e = hipSetDevice(g.device);
    if (e != hipSuccess) { delete c; return fail(VAEB_ERR_HIP, "hipSetDevice(%d): %s", g.device, hipGetErrorString(e)); }
    e = hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking);
    // Runtime switches (read here only; each alternative is a product path elsewhere or the
    // independent form an agreement test compares the default against -- DESIGN.md 4.4)
    if (const char* fb = getenv("VAEB_FOLD_BWD")) c->fold_bwd = atoi(fb) != 0;
    if (const char* bd = getenv("VAEB_BWD_DEFER")) c->bwd_defer = atoi(bd) != 0;
    if (const char* wd = getenv("VAEB_DW2_DEFER")) c->dw2_defer = atoi(wd) != 0;
    if (const char* ah = getenv("VAEB_ATOMIC_HO")) c->atomic_ho = atoi(ah) != 0 ? 1 : 0;
    if (const char* er = getenv("VAEB_ENC_RED")) c->enc_red = atoi(er) != 0 ? 1 : 0;
    if (const char* bk = getenv("VAEB_BF_FORK")) c->bf_fork = atoi(bk) != 0;
    if (const char* tt = getenv("VAEB_BF_DTT")) c->bf_dtt = atoi(tt) != 0;
    if (const char* zf = getenv("VAEB_BF_DZFUSE")) c->bf_dzfuse = atoi(zf) != 0;
    if (const char* bt = getenv("VAEB_BF_THIN")) c->bf_thin = atoi(bt) & 3;
    {
        const char* g8 = getenv("VAEB_BF_GEMM8");
        // default: the 8-phase loop for KC x KC (dhd), KC x KO (enc) and, since round 5, KO x KO
        // (the forked dW2 | dW6 and dW3): round 3 measured KO x KO on it slower (845 vs 816 us);
        // with the round-5 step (dz in dhd, the decoder on the 8-phase loop) it is faster:
        // 738.6 / 741.7 / 740.3 -> 726.8 / 728.7 / 727.4 us (profiles/r5/synth_ab.txt)
        g_gemm8 = g8 ? (int)strtol(g8, nullptr, 0) : 11;
    }
    if (e != hipSuccess) { delete c; return fail(VAEB_ERR_HIP, "stream/event create: %s", hipGetErrorString(e)); }
    const int64_t D = g.D, H = g.H, Z = g.Z;
    set_arena_layout(c);
    c->cap = std::max(r16(g.B), r16(c->c.max_eval_rows));
    const int64_t R = c->cap, RL = (int64_t)c->cap * g.L;
    int rc = 0;
    rc = rc ? rc : dalloc(&c->theta2[0], c->P);
    rc = rc ? rc : dalloc(&c->theta2[1], c->P);
    rc = rc ? rc : dalloc(&c->acc, c->P);
    rc = rc ? rc : dalloc(&c->grad, c->P + 1);
    if (g.estimator == VAEB_EST_FV || g.estimator == VAEB_EST_FVS) {
        rc = rc ? rc : dalloc(&c->fvmu, c->P);
        rc = rc ? rc : dalloc(&c->fvsg, c->P);
        rc = rc ? rc : dalloc(&c->fvam, c->P);
        rc = rc ? rc : dalloc(&c->fvas, c->P);
    }
    rc = rc ? rc : dalloc(&c->fv_part, kFvParts);
    rc = rc ? rc : dalloc(&c->xeval, (size_t)R * D);
    rc = rc ? rc : dalloc(&c->ictl, kCtlOrder + kOrderCap);
    rc = rc ? rc : dalloc(&c->step, 1);
    rc = rc ? rc : dalloc(&c->eval_acc, 2);
    rc = rc ? rc : dalloc(&c->h, (size_t)R * H);
    rc = rc ? rc : dalloc(&c->mu, (size_t)R * Z);
    rc = rc ? rc : dalloc(&c->lv, (size_t)R * Z);
    rc = rc ? rc : dalloc(&c->eps, (size_t)RL * Z);
    rc = rc ? rc : dalloc(&c->z, (size_t)RL * Z);
    rc = rc ? rc : dalloc(&c->hd, (size_t)RL * H);
    rc = rc ? rc : dalloc(&c->y, (size_t)RL * D);
    // dA6 directly after dA2: the dhd loaders address both through one descriptor (PDhdT)
    rc = rc ? rc : dalloc(&c->dA2, (size_t)RL * D * (gaussian(c) ? 2 : 1));
    if (!rc && gaussian(c)) c->dA6 = c->dA2 + (size_t)RL * D;
    rc = rc ? rc : dalloc(&c->dA1, (size_t)RL * H);
    rc = rc ? rc : dalloc(&c->dZ, (size_t)RL * Z);
    rc = rc ? rc : dalloc(&c->dMuLv, (size_t)R * 2 * Z);
    rc = rc ? rc : dalloc(&c->dA3, (size_t)R * H);
    rc = rc ? rc : dalloc(&c->kl_part, (size_t)RL * cdiv(Z, 16));
    rc = rc ? rc : dalloc(&c->lp_part, (size_t)RL * cdiv(D, 16));
    {   // folded-latent slabs and arrival counters (training minibatch only)
        const int64_t Bp = r16(g.B), nctH = cdiv(H, 16);
        rc = rc ? rc : dalloc(&c->slab_ml, (size_t)(Bp * nctH * 64));
        rc = rc ? rc : dalloc(&c->slab_dz, (size_t)(g.L * Bp * nctH * 32));
        rc = rc ? rc : dalloc(&c->cnt_ml, (size_t)(Bp / 16));
        rc = rc ? rc : dalloc(&c->cnt_dz, (size_t)std::max<int64_t>(Bp / 16, kLatCnt * kLatCntStride));
        rc = rc ? rc : dalloc(&c->w2pend, 1);
        // one allocation: the guard word the contributors set sits at acc_ml[-1] (latent.hpp fx_inc)
        const size_t nacc = (size_t)(Bp * 2 * Z * kFxStride);
        rc = rc ? rc : dalloc(&c->blk, kBlkAcc + 2 * nacc);
        if (!rc) {
            c->epoch = reinterpret_cast<double*>(c->blk);
            c->elbo_out = reinterpret_cast<float*>(c->blk + kBlkElbo);
            c->acc_ml = c->blk + kBlkAcc;
            c->acc_dz = c->acc_ml + nacc;
        }
    }
    if (!rc && is_bf16(c)) rc = bf_alloc(c);
    if (!rc && is_bf16(c)) {
        if (hipStreamCreateWithFlags(&c->s3, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->fk_ev[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->fk_ev[1], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->fk_ev[2], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->fk_ev[3], hipEventDisableTiming) != hipSuccess)
            rc = fail(VAEB_ERR_HIP, "fork stream / events");
    }
    if (rc) { vaeb_destroy(c); return rc; }
    if (hipHostMalloc((void**)&c->h_ctl, sizeof(int) * (kCtlOrder + kOrderCap), 0) != hipSuccess ||
        hipHostMalloc((void**)&c->h_elbo, sizeof(float) * 4, 0) != hipSuccess ||
        hipHostMalloc((void**)&c->h_d2, sizeof(double) * 4, 0) != hipSuccess) {
        vaeb_destroy(c);
        return fail(VAEB_ERR_NOMEM, "hipHostMalloc failed");
    }
    {
        // the step's scalar result written by the GPU straight into mapped, coherent host
        // memory: vaeb_update reads it with no device -> host copy (and no stream sync)
        void* dp = nullptr;
        if (hipHostMalloc((void**)&c->h_out, sizeof(float) * 4, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer(&dp, c->h_out, 0) != hipSuccess) {
            vaeb_destroy(c);
            return fail(VAEB_ERR_NOMEM, "mapped host ELBO slot");
        }
        memset(c->h_out, 0, sizeof(float) * 4);
        c->elbo_out = static_cast<float*>(dp);
    }
    hipEventCreateWithFlags(&c->ctl_ev, hipEventDisableTiming);
    hipEventRecord(c->ctl_ev, c->s);
    for (auto& ev : c->pev) hipEventCreate(&ev);
    if (hipDeviceSynchronize() != hipSuccess) { vaeb_destroy(c); return fail(VAEB_ERR_HIP, "device init failed"); }
    *out = c;
    return 0;
}

int vaeb_destroy(vaeb_ctx* c) {
    if (!c) return 0;
    if (c->s) hipStreamSynchronize(c->s);
    if (c->s2) hipStreamSynchronize(c->s2);
    if (c->s3) hipStreamSynchronize(c->s3);
    free_graphs(c);
    bf_free(c);
    if (c->comm) ncclCommDestroy(c->comm);
    float* fp[] = {c->theta2[0], c->theta2[1], c->acc, c->grad, c->fvmu, c->fvsg, c->fvam, c->fvas, c->fv_part, c->data, c->xeval, c->xval,
                   c->eps_in, c->h, c->mu, c->lv, c->eps, c->z, c->hd, c->y, c->dA2, c->dA1,   // dA6 lives in dA2's block
                   c->dZ, c->dMuLv, c->dA3, c->kl_part, c->lp_part, c->slab_ml, c->slab_dz, c->yacc,
                   c->fvzeta};
    for (float* p : fp) if (p) hipFree(p);
    if (c->cnt_ml) hipFree(c->cnt_ml);
    if (c->cnt_dz) hipFree(c->cnt_dz);
    if (c->blk) hipFree(c->blk);   // epoch, elbo_out, acc_ml, acc_dz live in it
    if (c->ictl) hipFree(c->ictl);
    if (c->step) hipFree(c->step);
    if (c->eval_acc) hipFree(c->eval_acc);
    if (c->h_ctl) hipHostFree(c->h_ctl);
    if (c->h_elbo) hipHostFree(c->h_elbo);
    if (c->h_out) hipHostFree(c->h_out);
    if (c->h_d2) hipHostFree(c->h_d2);
    if (c->ctl_ev) hipEventDestroy(c->ctl_ev);
    for (auto& ev : c->pev) if (ev) hipEventDestroy(ev);
    for (auto& ev : c->dp_ev) if (ev) hipEventDestroy(ev);
    for (auto& ev : c->fk_ev) if (ev) hipEventDestroy(ev);
    if (c->s3) hipStreamDestroy(c->s3);
    if (c->s2) hipStreamDestroy(c->s2);
    if (c->s) hipStreamDestroy(c->s);
    delete c;
    return 0;
}

int vaeb_num_params(const vaeb_ctx* c, int64_t* n) {
    if (!c || !n) return fail(VAEB_ERR_ARG, "null argument");
    *n = c->P;
    return 0;
}

int vaeb_set_data(vaeb_ctx* c, const float* x, int64_t n_rows) {
    if (!c || !x || n_rows <= 0) return fail(VAEB_ERR_ARG, "bad data arguments");
    HIP_TRY(hipStreamSynchronize(c->s));
    if (c->data) { hipFree(c->data); c->data = nullptr; }
    free_graphs(c);  // graphs hold the data pointer
    c->graph_failed = false;
    if (is_bf16(c)) {
        // the bf16 engine keeps only a bf16 copy; c->data stays a 16-byte placeholder
        if (c->bf.x) { hipFree(c->bf.x); c->bf.x = nullptr; }
        if (c->bf.xbits) { hipFree(c->bf.xbits); c->bf.xbits = nullptr; }
        // a binary dataset (every value exactly 0 or 1) also as bits, for the Bernoulli decoder
        // epilogue's x tile (EpiDecOutT::load_in): 1/16 of its bytes, the same values
        const int64_t D = c->c.D, nel = n_rows * D;
        bool binary = D % 32 == 0;
        for (int64_t i = 0; binary && i < nel; ++i) binary = x[i] == 0.f || x[i] == 1.f;
        if (binary) {
            std::vector<uint32_t> bits((size_t)(nel / 32), 0u);
            for (int64_t i = 0; i < nel; ++i)
                if (x[i] != 0.f) bits[(size_t)(i >> 5)] |= 1u << (i & 31);
            if (int rc = dalloc(&c->bf.xbits, bits.size())) return rc;
            HIP_TRY(hipMemcpy(c->bf.xbits, bits.data(), sizeof(uint32_t) * bits.size(), hipMemcpyHostToDevice));
        }
        if (int rc = dalloc(&c->bf.x, (size_t)n_rows * c->c.D)) return rc;
        if (int rc = dalloc(&c->data, 4)) return rc;
        if (int rc = bf_upload_rows(c, x, n_rows, c->bf.x)) return rc;
        HIP_TRY(hipStreamSynchronize(c->s));
        c->nrows = n_rows;
        return 0;
    }
    if (int rc = dalloc(&c->data, (size_t)n_rows * c->c.D)) return rc;
    HIP_TRY(hipMemcpy(c->data, x, sizeof(float) * (size_t)n_rows * c->c.D, hipMemcpyHostToDevice));
    c->nrows = n_rows;
    return 0;
}

static int xfer(vaeb_ctx* c, float* dev, const float* hin, float* hout, int64_t n, int64_t want) {
    if (!c || (!hin && !hout)) return fail(VAEB_ERR_ARG, "null argument");
    if (!dev) return fail(VAEB_ERR_STATE, "state not allocated for this estimator");
    if (n != want) return fail(VAEB_ERR_ARG, "size mismatch: got %lld, expected %lld", (long long)n, (long long)want);
    if (int rc = w2_flush(c)) return rc;   // a pending deferred dW2 first: the state is whole
    HIP_TRY(hipStreamSynchronize(c->s));
    if (hin) HIP_TRY(hipMemcpy(dev, hin, sizeof(float) * n, hipMemcpyHostToDevice));
    else HIP_TRY(hipMemcpy(hout, dev, sizeof(float) * n, hipMemcpyDeviceToHost));
    return 0;
}

int vaeb_set_params(vaeb_ctx* c, const float* f, int64_t n) {
    if (int rc = xfer(c, c ? c->theta2[c->par] : nullptr, f, nullptr, n, c ? c->P : 0)) return rc;
    if (is_bf16(c)) {
        if (int rc = bf_make_shadow(c, c->par)) return rc;
        HIP_TRY(hipStreamSynchronize(c->s));
    }
    return 0;
}
int vaeb_get_params(vaeb_ctx* c, float* f, int64_t n) { return xfer(c, c ? c->theta2[c->par] : nullptr, nullptr, f, n, c ? c->P : 0); }
int vaeb_set_adagrad_state(vaeb_ctx* c, const float* f, int64_t n) { return xfer(c, c ? c->acc : nullptr, f, nullptr, n, c ? c->P : 0); }
int vaeb_get_adagrad_state(vaeb_ctx* c, float* f, int64_t n) {
    if (c) if (int rc = dp_gather_acc(c)) return rc;   // sharded DP: a collective (every rank calls)
    return xfer(c, c ? c->acc : nullptr, nullptr, f, n, c ? c->P : 0);
}
int vaeb_get_grads(vaeb_ctx* c, float* f, int64_t n) { return xfer(c, c ? c->grad : nullptr, nullptr, f, n, c ? c->P : 0); }

int vaeb_set_fv_state(vaeb_ctx* c, const float* mu, const float* sg, const float* am, const float* as, int64_t n) {
    int rc = 0;
    rc = rc ? rc : xfer(c, c ? c->fvmu : nullptr, mu, nullptr, n, c ? c->P : 0);
    rc = rc ? rc : xfer(c, c ? c->fvsg : nullptr, sg, nullptr, n, c ? c->P : 0);
    rc = rc ? rc : xfer(c, c ? c->fvam : nullptr, am, nullptr, n, c ? c->P : 0);
    rc = rc ? rc : xfer(c, c ? c->fvas : nullptr, as, nullptr, n, c ? c->P : 0);
    return rc;
}

int vaeb_get_fv_state(vaeb_ctx* c, float* mu, float* sg, float* am, float* as, int64_t n) {
    int rc = 0;
    rc = rc ? rc : xfer(c, c ? c->fvmu : nullptr, nullptr, mu, n, c ? c->P : 0);
    rc = rc ? rc : xfer(c, c ? c->fvsg : nullptr, nullptr, sg, n, c ? c->P : 0);
    rc = rc ? rc : xfer(c, c ? c->fvam : nullptr, nullptr, am, n, c ? c->P : 0);
    rc = rc ? rc : xfer(c, c ? c->fvas : nullptr, nullptr, as, n, c ? c->P : 0);
    return rc;
}

int vaeb_set_eps_mode(vaeb_ctx* c, int32_t mode, uint64_t seed) {
    if (!c || (mode != VAEB_EPS_PHILOX && mode != VAEB_EPS_HOST)) return fail(VAEB_ERR_ARG, "bad eps mode");
    HIP_TRY(hipStreamSynchronize(c->s));
    // captured steps hold the eps mode's kernels and the Philox seed by value (make_args)
    if (mode != c->eps_mode || seed != c->seed) { free_graphs(c); c->graph_failed = false; }
    c->eps_mode = mode;
    c->seed = seed;
    return 0;
}

int vaeb_push_eps(vaeb_ctx* c, const float* eps, int64_t rows, int32_t L) {
    if (!c || !eps || rows <= 0) return fail(VAEB_ERR_ARG, "bad eps arguments");
    if (L != c->c.L) return fail(VAEB_ERR_ARG, "eps L=%d does not match the model L=%d", L, c->c.L);
    const int64_t n = rows * L * c->c.Z;
    HIP_TRY(hipStreamSynchronize(c->s));
    if (n > c->eps_in_cap) {
        if (c->eps_in) hipFree(c->eps_in);
        c->eps_in = nullptr;
        free_graphs(c);
        c->graph_failed = false;
        if (int rc = dalloc(&c->eps_in, (size_t)n)) return rc;
        c->eps_in_cap = n;
    }
    if (rows != c->eps_rows) { free_graphs(c); c->graph_failed = false; }
    c->eps_rows = rows;
    HIP_TRY(hipMemcpy(c->eps_in, eps, sizeof(float) * n, hipMemcpyHostToDevice));
    return 0;
}

int vaeb_push_fv_noise(vaeb_ctx* c, const float* zeta, int64_t n) {
    if (!c || !zeta) return fail(VAEB_ERR_ARG, "null argument");
    if (c->c.estimator != VAEB_EST_FVS) return fail(VAEB_ERR_STATE, "weight noise is for the VAEB_EST_FVS estimator");
    if (n != c->P) return fail(VAEB_ERR_ARG, "weight noise needs %lld values (got %lld)", (long long)c->P, (long long)n);
    HIP_TRY(hipStreamSynchronize(c->s));
    if (!c->fvzeta) {
        if (int rc = dalloc(&c->fvzeta, (size_t)c->P)) return rc;
        free_graphs(c);   // captured steps hold the noise pointer
        c->graph_failed = false;
    }
    HIP_TRY(hipMemcpy(c->fvzeta, zeta, sizeof(float) * (size_t)n, hipMemcpyHostToDevice));
    return 0;
}

int vaeb_set_step(vaeb_ctx* c, int64_t step) {
    if (!c) return fail(VAEB_ERR_ARG, "null ctx");
    HIP_TRY(hipStreamSynchronize(c->s));
    HIP_TRY(hipMemcpy(c->step, &step, sizeof(step), hipMemcpyHostToDevice));
    return 0;
}

static int host_eps_ready(vaeb_ctx* c, int64_t rows) {
    if (c->eps_mode == VAEB_EPS_HOST && c->eps_rows != rows)
        return fail(VAEB_ERR_STATE, "host eps mode: pushed %lld rows, step needs %lld (call vaeb_push_eps)",
                    (long long)c->eps_rows, (long long)rows);
    return 0;
}

// Wait until the step's last kernel has written [SGVB / B, flags] into the mapped host slot
// (kernels_aux.hpp elbo_store: flags = 2 | status), polling the slot; the stream is queried
// now and then so that a failed or already-finished stream ends the wait.
static int wait_step_result(vaeb_ctx* c) {
    volatile uint32_t* flag = reinterpret_cast<volatile uint32_t*>(&c->h_out[1]);
    for (uint64_t spin = 0; *flag == 0u; ++spin) {
        if ((spin & 255) == 255) {
            const hipError_t q = hipStreamQuery(c->s);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return fail(VAEB_ERR_HIP, "step failed: %s", hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
    if (*flag == 0u) return fail(VAEB_ERR_STATE, "internal: the step wrote no result");
    return 0;
}

// The sticky step status read at a sync point (kernels_aux.hpp elbo_emit): cleared, and
// reported as VAEB_ERR_NUMERIC.
static int take_status(vaeb_ctx* c, uint64_t st) {
    if (!st) return 0;
    HIP_TRY(hipMemsetAsync(c->blk + kBlkStatus, 0, sizeof(uint64_t), c->s));
    HIP_TRY(hipStreamSynchronize(c->s));
    return fail(VAEB_ERR_NUMERIC, "the step overflowed the fixed-point latent hand-off (a partial outside +-2^17, "
                                  "NaN or inf): its latent values are NaN");
}

int vaeb_update(vaeb_ctx* c, int32_t batch_index, float* out) {
    if (!c) return fail(VAEB_ERR_ARG, "null ctx");
    if (int rc = check_batches(c, &batch_index, 1)) return rc;
    if (int rc = host_eps_ready(c, c->c.B)) return rc;
    // The reference calls update() once per minibatch and waits for its value (VAEB.py:
    // 577-579).  That call is ONE eager step whose minibatch index rides the launch
    // arguments (no order upload, no graph launch), and its value is read from the mapped
    // host slot the step's last kernel writes: 65 -> ~55 us per call (scripts/call_ab.py).
    // Steps still queued from vaeb_update_many / vaeb_update_async would write the mapped
    // slot too: drain them first, so the value read below is this call's step.
    if (c->async_pending) {
        HIP_TRY(hipStreamSynchronize(c->s));
        c->async_pending = false;
    }
    volatile uint32_t* flag = reinterpret_cast<volatile uint32_t*>(&c->h_out[1]);
    *flag = 0u;
    if (int rc = step_eager(c, batch_index)) return rc;
    if (int rc = wait_step_result(c)) return rc;
    if (out) *out = c->h_out[0];
    return take_status(c, *flag & 1u);
}

int vaeb_update_many(vaeb_ctx* c, const int32_t* idx, int32_t n) {
    if (!c || (!idx && n > 0) || n < 0) return fail(VAEB_ERR_ARG, "bad arguments");
    if (int rc = check_batches(c, idx, n)) return rc;
    if (int rc = host_eps_ready(c, c->c.B)) return rc;
    // host eps holds ONE step's noise: a multi-step call would train every step on it
    if (c->eps_mode == VAEB_EPS_HOST && n > 1)
        return fail(VAEB_ERR_STATE, "host eps mode: one step per call (push eps before each vaeb_update)");
    if (n > 0) c->async_pending = true;
    // the call's first step goes out eagerly with its minibatch index in the launch arguments
    // (it reads no order and no cursor): the GPU runs it while the host submits the graph of
    // the remaining steps (which would otherwise lead every call).  The order of those steps
    // is uploaded right behind the step's first launch (order_hook): launched after the whole
    // eager step it started ~6 us after the GPU had finished the step, launched before it the
    // step's first kernel started ~4.5 us after the upload (kernel traces,
    // profiles/r6/call_timeline.txt)
    const bool eager = n >= 2 && c->c.use_graph && c->gN[0][1] && !c->graph_failed && flips(c);
    for (int32_t done = eager ? 1 : 0; done < n;) {
        const int32_t m = std::min<int32_t>(n - done, kOrderCap);
        if (eager && done == 1) {
            if (m <= kArgOrder) {   // the upload rides behind the eager step's first launch
                c->order_pend.n = m;
                memcpy(c->order_pend.v, idx + done, sizeof(int) * (size_t)m);
                c->order_pending = true;
            } else if (int rc = upload_order(c, idx + done, m)) {
                return rc;
            }
            const int rc = step_eager(c, idx[0]);
            const int rh = order_hook(c);   // where the step's launch path took no hook
            if (rc) return rc;
            if (rh) return rh;
        } else if (int rc = upload_order(c, idx + done, m)) {
            return rc;
        }
        if (int rc = run_steps(c, m)) return rc;
        done += m;
    }
    return 0;
}

int vaeb_update_async(vaeb_ctx* c, int32_t batch_index) { return vaeb_update_many(c, &batch_index, 1); }

int vaeb_epoch_elbo(vaeb_ctx* c, double* out_sum, int64_t* out_steps) {
    if (!c) return fail(VAEB_ERR_ARG, "null ctx");
    // epoch sums and the sticky status in one copy, then all three cleared
    HIP_TRY(hipMemcpyAsync(c->h_d2, c->epoch, 3 * sizeof(double), hipMemcpyDeviceToHost, c->s));
    HIP_TRY(hipMemsetAsync(c->epoch, 0, 3 * sizeof(double), c->s));
    HIP_TRY(hipStreamSynchronize(c->s));
    c->async_pending = false;
    if (out_sum) *out_sum = c->h_d2[0];
    if (out_steps) *out_steps = (int64_t)c->h_d2[1];
    uint64_t st;
    memcpy(&st, &c->h_d2[2], sizeof(st));
    return st ? fail(VAEB_ERR_NUMERIC, "a step since the last read overflowed the fixed-point latent hand-off "
                                       "(a partial outside +-2^17, NaN or inf): its latent values are NaN")
              : 0;
}

int vaeb_synchronize(vaeb_ctx* c) {
    if (!c) return fail(VAEB_ERR_ARG, "null ctx");
    HIP_TRY(hipStreamSynchronize(c->s));
    c->async_pending = false;
    return 0;
}

// Forward-only passes in device chunks (validate / reconstruct).  The arena the data term
// reads: the current theta, or for VAEB_EST_FVS the posterior mean mu_theta (copied into
// the spare arena once per call).
static int eval_arena(vaeb_ctx* c, int* epar) {
    if (int rc = w2_flush(c)) return rc;
    *epar = c->par;
    if (c->c.estimator == VAEB_EST_FVS) {
        *epar = c->par ^ 1;
        HIP_TRY(hipMemcpyAsync(c->theta2[*epar], c->fvmu, sizeof(float) * (size_t)c->P, hipMemcpyDeviceToDevice, c->s));
    }
    return 0;
}

// One fp32 chunk: `rows` device rows at x = global rows [r0, r0 + rows).  MODE_EVAL adds
// the chunk's SGVB into eval_acc; MODE_RECON copies the decoder means to out_y (host).
static int eval_chunk_f32(vaeb_ctx* c, int epar, const float* x, int rows, int64_t r0, int mode, float* out_y,
                          float* out_lv = nullptr) {
    const vaeb_config& g = c->c;
    StepArgs a = make_args(c, epar, rows, mode, x, false);
    a.row_base_add = r0;
    a.eps_in = c->eps_in ? c->eps_in + r0 * g.Z : nullptr;
    a.eps_in_ld = c->eps_rows;
    Prof pr{c, false};
    if (int rc = enqueue_forward(c, a, pr)) return rc;
    if (mode == MODE_RECON) {
        HIP_TRY(hipMemcpyAsync(out_y, c->y, sizeof(float) * (size_t)rows * g.D, hipMemcpyDeviceToHost, c->s));
        if (out_lv)
            HIP_TRY(hipMemcpyAsync(out_lv, c->dA6, sizeof(float) * (size_t)rows * g.D, hipMemcpyDeviceToHost, c->s));
    } else {
        ElboArgs e = base_elbo(c, a);
        e.eval_acc = c->eval_acc;
        hipLaunchKernelGGL(elbo_kernel, dim3(1), dim3(256), 0, c->s, e);
        CHECK_LAUNCH();
    }
    return 0;
}

// SGVB of n evaluated rows from eval_acc (after an optional all-reduce of it over the
// ranks); the FV estimators add thetaPrior: x.shape[0] * (sum logp + sum KL) + thetaPrior
// (VAEB.py:364).
static int eval_finish(vaeb_ctx* c, int64_t n, bool allreduce, double* out_sum) {
    const vaeb_config& g = c->c;
    double tp = 0.0;
    const bool fvx = g.estimator == VAEB_EST_FV || g.estimator == VAEB_EST_FVS;
    if (fvx) {
        hipLaunchKernelGGL(fv_kernel, dim3(kFvParts), dim3(256), 0, c->s, c->fvmu, c->fvsg, c->fvam, c->fvas, c->P,
                           g.lr, g.adagrad_eps, 0, c->fv_part);
        CHECK_LAUNCH();
        std::vector<float> parts(kFvParts);
        HIP_TRY(hipMemcpyAsync(parts.data(), c->fv_part, sizeof(float) * kFvParts, hipMemcpyDeviceToHost, c->s));
        HIP_TRY(hipStreamSynchronize(c->s));
        for (float p : parts) tp += p;
    }
    if (allreduce && c->comm) {
        ncclResult_t r = ncclAllReduce(c->eval_acc, c->eval_acc, 1, ncclDouble, ncclSum, c->comm, c->s);
        if (r != ncclSuccess) return fail(VAEB_ERR_COMM, "ncclAllReduce(validation): %s", ncclGetErrorString(r));
    }
    HIP_TRY(hipMemcpyAsync(c->h_d2, c->eval_acc, 2 * sizeof(double), hipMemcpyDeviceToHost, c->s));
    HIP_TRY(hipStreamSynchronize(c->s));
    const double data = c->h_d2[0];
    *out_sum = fvx ? (double)n * data + tp : data;
    return 0;
}

// Host rows: each chunk is staged through xeval (stream-ordered, one sync at the end).
static int eval_rows(vaeb_ctx* c, const float* x, int64_t n, int mode, float* out_y, double* out_sum,
                     float* out_lv = nullptr) {
    if (!c || !x || n <= 0) return fail(VAEB_ERR_ARG, "bad arguments");
    if (mode == MODE_EVAL && c->eps_mode == VAEB_EPS_HOST && c->eps_rows != n)
        return fail(VAEB_ERR_STATE, "host eps mode: validate needs eps for %lld rows (pushed %lld)", (long long)n,
                    (long long)c->eps_rows);
    const vaeb_config& g = c->c;
    const int chunk = c->c.max_eval_rows;
    HIP_TRY(hipMemsetAsync(c->eval_acc, 0, 2 * sizeof(double), c->s));
    int epar = c->par;
    if (!is_bf16(c)) if (int rc = eval_arena(c, &epar)) return rc;
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
        const int rows = (int)std::min<int64_t>(chunk, n - r0);
        float* yo = out_y ? out_y + r0 * g.D : nullptr;
        if (is_bf16(c)) {
            if (int rc = bf_eval_chunk(c, x + r0 * g.D, rows, r0, mode, yo)) return rc;
            continue;
        }
        HIP_TRY(hipMemcpyAsync(c->xeval, x + r0 * g.D, sizeof(float) * (size_t)rows * g.D, hipMemcpyHostToDevice, c->s));
        if (int rc = eval_chunk_f32(c, epar, c->xeval, rows, r0, mode, yo, out_lv ? out_lv + r0 * g.D : nullptr))
            return rc;
    }
    if (mode == MODE_EVAL) return eval_finish(c, n, false, out_sum);
    HIP_TRY(hipStreamSynchronize(c->s));
    return 0;
}

int vaeb_validate(vaeb_ctx* c, const float* x, int64_t n, double* out_sum) {
    if (!out_sum) return fail(VAEB_ERR_ARG, "null out_sum");
    return eval_rows(c, x, n, MODE_EVAL, nullptr, out_sum);
}

int vaeb_set_valid_data(vaeb_ctx* c, const float* x, int64_t n) {
    if (!c || !x || n <= 0) return fail(VAEB_ERR_ARG, "bad validation-set arguments");
    HIP_TRY(hipStreamSynchronize(c->s));
    if (c->xval) { hipFree(c->xval); c->xval = nullptr; }
    if (c->bf.xval) { hipFree(c->bf.xval); c->bf.xval = nullptr; }
    c->nval = 0;
    if (is_bf16(c)) {
        if (int rc = dalloc(&c->bf.xval, (size_t)n * c->c.D)) return rc;
        if (int rc = bf_upload_rows(c, x, n, c->bf.xval)) return rc;
        HIP_TRY(hipStreamSynchronize(c->s));
    } else {
        if (int rc = dalloc(&c->xval, (size_t)n * c->c.D)) return rc;
        HIP_TRY(hipMemcpy(c->xval, x, sizeof(float) * (size_t)n * c->c.D, hipMemcpyHostToDevice));
    }
    c->nval = n;
    return 0;
}

// This rank's contiguous share of the resident rows: the first (n % world) ranks take one
// extra row (the row split of vaeb_amd/dp.py).
static void valid_share(const vaeb_ctx* c, int64_t* lo, int64_t* rows) {
    const int64_t W = c->comm ? c->world : 1, r = c->comm ? c->rank : 0;
    const int64_t base = c->nval / W, extra = c->nval % W;
    *rows = base + (r < extra ? 1 : 0);
    *lo = r * base + std::min<int64_t>(r, extra);
}

int vaeb_validate_resident(vaeb_ctx* c, double* out_sum) {
    if (!c || !out_sum) return fail(VAEB_ERR_ARG, "null argument");
    if (c->nval <= 0) return fail(VAEB_ERR_STATE, "vaeb_set_valid_data has not been called");
    if (c->eps_mode == VAEB_EPS_HOST && c->eps_rows != c->nval)
        return fail(VAEB_ERR_STATE, "host eps mode: resident validation needs eps for all %lld rows (pushed %lld)",
                    (long long)c->nval, (long long)c->eps_rows);
    const vaeb_config& g = c->c;
    int64_t lo = 0, rows = 0;
    valid_share(c, &lo, &rows);
    HIP_TRY(hipMemsetAsync(c->eval_acc, 0, 2 * sizeof(double), c->s));
    int epar = c->par;
    if (!is_bf16(c)) if (int rc = eval_arena(c, &epar)) return rc;
    const int chunk = g.max_eval_rows;
    for (int64_t r0 = lo; r0 < lo + rows; r0 += chunk) {
        const int m = (int)std::min<int64_t>(chunk, lo + rows - r0);
        if (is_bf16(c)) {
            if (int rc = bf_eval_chunk_dev(c, c->bf.xval + r0 * g.D, m, r0, MODE_EVAL, nullptr)) return rc;
        } else {
            if (int rc = eval_chunk_f32(c, epar, c->xval + r0 * g.D, m, r0, MODE_EVAL, nullptr)) return rc;
        }
    }
    return eval_finish(c, c->nval, true, out_sum);
}

int vaeb_get_step(vaeb_ctx* c, int64_t* step) {
    if (!c || !step) return fail(VAEB_ERR_ARG, "null argument");
    HIP_TRY(hipStreamSynchronize(c->s));
    HIP_TRY(hipMemcpy(step, c->step, sizeof(int64_t), hipMemcpyDeviceToHost));
    return 0;
}

int vaeb_comm_count(vaeb_ctx* c, int32_t* out_world) {
    if (!c || !out_world) return fail(VAEB_ERR_ARG, "null argument");
    if (!c->comm) { *out_world = 1; return 0; }
    int n = 0;
    ncclResult_t r = ncclCommCount(c->comm, &n);
    if (r != ncclSuccess) return fail(VAEB_ERR_COMM, "ncclCommCount: %s", ncclGetErrorString(r));
    *out_world = n;
    return 0;
}

// ------------------------------------------------------------------ native checkpoint
namespace {
struct CkptHeader {
    char magic[8];          // "VAEBCKPT"
    int32_t version;        // 1
    int32_t D, H, Z, L, decoder, estimator, objective, dtype;
    int32_t eps_mode, has_fv;
    int64_t P;
    uint64_t seed;
    int64_t step;
    int64_t reserved[4];
};
constexpr char kCkptMagic[8] = {'V', 'A', 'E', 'B', 'C', 'K', 'P', 'T'};

struct FileCloser { FILE* f; ~FileCloser() { if (f) fclose(f); } };
}  // namespace

int vaeb_checkpoint_save(vaeb_ctx* c, const char* path) {
    if (!c) return fail(VAEB_ERR_ARG, "null argument");
    // path NULL: a non-writing rank of a multi-rank communicator joining the gather;
    // anywhere else it is a caller error, reported before anything runs
    if (!path && !(c->comm && c->world > 1))
        return fail(VAEB_ERR_ARG, "checkpoint: null path (only a non-writing rank of a multi-rank communicator passes NULL)");
    if (int rc = w2_flush(c)) return rc;   // a pending deferred dW2 (vaeb_ctx::dw2_defer)
    if (int rc = dp_gather_acc(c)) return rc;   // sharded DP: the whole Adagrad state (every rank calls)
    if (!path) return 0;
    const vaeb_config& g = c->c;
    CkptHeader h{};
    memcpy(h.magic, kCkptMagic, 8);
    h.version = 1;
    h.D = g.D; h.H = g.H; h.Z = g.Z; h.L = g.L;
    h.decoder = g.decoder; h.estimator = g.estimator; h.objective = g.objective; h.dtype = g.dtype;
    h.eps_mode = c->eps_mode;
    h.has_fv = c->fvmu ? 1 : 0;
    h.P = c->P;
    h.seed = c->seed;
    HIP_TRY(hipStreamSynchronize(c->s));
    HIP_TRY(hipMemcpy(&h.step, c->step, sizeof(int64_t), hipMemcpyDeviceToHost));
    std::vector<float*> arrs = {c->theta2[c->par], c->acc};
    if (h.has_fv) arrs.insert(arrs.end(), {c->fvmu, c->fvsg, c->fvam, c->fvas});
    std::vector<float> buf((size_t)c->P);
    FileCloser fc{fopen(path, "wb")};
    if (!fc.f) return fail(VAEB_ERR_ARG, "checkpoint: cannot open %s for writing", path);
    if (fwrite(&h, sizeof(h), 1, fc.f) != 1) return fail(VAEB_ERR_ARG, "checkpoint: write failed (%s)", path);
    for (float* d : arrs) {
        HIP_TRY(hipMemcpy(buf.data(), d, sizeof(float) * buf.size(), hipMemcpyDeviceToHost));
        if (fwrite(buf.data(), sizeof(float), buf.size(), fc.f) != buf.size())
            return fail(VAEB_ERR_ARG, "checkpoint: write failed (%s)", path);
    }
    if (fflush(fc.f) != 0) return fail(VAEB_ERR_ARG, "checkpoint: flush failed (%s)", path);
    return 0;
}

int vaeb_checkpoint_load(vaeb_ctx* c, const char* path) {
    if (!c || !path) return fail(VAEB_ERR_ARG, "null argument");
    if (int rc = w2_flush(c)) return rc;   // a pending deferred dW2 (vaeb_ctx::dw2_defer)
    const vaeb_config& g = c->c;
    FileCloser fc{fopen(path, "rb")};
    if (!fc.f) return fail(VAEB_ERR_ARG, "checkpoint: cannot open %s", path);
    CkptHeader h{};
    if (fread(&h, sizeof(h), 1, fc.f) != 1 || memcmp(h.magic, kCkptMagic, 8) != 0 || h.version != 1)
        return fail(VAEB_ERR_ARG, "checkpoint: %s is not a version-1 vaeb checkpoint", path);
    if (h.objective != g.objective || h.dtype != g.dtype)
        return fail(VAEB_ERR_ARG, "checkpoint: %s was written by an objective=%d dtype=%d context, this one is "
                    "objective=%d dtype=%d", path, h.objective, h.dtype, g.objective, g.dtype);
    if (h.D != g.D || h.H != g.H || h.Z != g.Z || h.L != g.L || h.decoder != g.decoder ||
        h.estimator != g.estimator || h.P != c->P)
        return fail(VAEB_ERR_ARG, "checkpoint: %s holds a %d-%d-%d L=%d dec=%d est=%d model, the context is "
                    "%d-%d-%d L=%d dec=%d est=%d", path, h.D, h.H, h.Z, h.L, h.decoder, h.estimator,
                    g.D, g.H, g.Z, g.L, g.decoder, g.estimator);
    if (h.has_fv && !c->fvmu) return fail(VAEB_ERR_ARG, "checkpoint: variational state without an FV context");
    std::vector<float> buf((size_t)c->P);
    std::vector<float*> arrs = {c->theta2[c->par], c->acc};
    if (h.has_fv) arrs.insert(arrs.end(), {c->fvmu, c->fvsg, c->fvam, c->fvas});
    HIP_TRY(hipStreamSynchronize(c->s));
    for (float* d : arrs) {
        if (fread(buf.data(), sizeof(float), buf.size(), fc.f) != buf.size())
            return fail(VAEB_ERR_ARG, "checkpoint: %s is truncated", path);
        HIP_TRY(hipMemcpy(d, buf.data(), sizeof(float) * buf.size(), hipMemcpyHostToDevice));
    }
    if (is_bf16(c)) {
        if (int rc = bf_make_shadow(c, c->par)) return rc;
        HIP_TRY(hipStreamSynchronize(c->s));
    }
    HIP_TRY(hipMemcpy(c->step, &h.step, sizeof(int64_t), hipMemcpyHostToDevice));
    // captured steps hold the eps mode's kernels and the Philox seed by value (make_args)
    if (h.eps_mode != c->eps_mode || h.seed != c->seed) { free_graphs(c); c->graph_failed = false; }
    c->eps_mode = h.eps_mode;
    c->seed = h.seed;
    return 0;
}

int vaeb_reconstruct(vaeb_ctx* c, const float* x, int64_t n, float* out_y) {
    return vaeb_reconstruct_full(c, x, n, 0, out_y, nullptr);
}

int vaeb_reconstruct_sampled(vaeb_ctx* c, const float* x, int64_t n, int32_t n_samples, float* out_y) {
    return vaeb_reconstruct_full(c, x, n, n_samples, out_y, nullptr);
}

// VAEB.reconstruct (VAEB.py:267-291) before its closing multivariate_normal draw: the
// decoder outputs at z = mu (n_samples <= 0) or averaged over n_samples posterior draws
// z_s = mu + exp(lv / 2) eps_s, summed on device in sample order (:279-291).  eps_s:
// Philox stream s + 1 of the validation domain, or (host eps mode) rows [s * n, (s + 1) * n)
// of the pushed eps.  out_lv (Gaussian decoder, fp32 engine): the log-sigma head, averaged
// the same way (:284, 289) -- the caller's draw is y_mu + exp(y_log_sigma) * N(0, 1) (:295-297).
int vaeb_reconstruct_full(vaeb_ctx* c, const float* x, int64_t n, int32_t n_samples, float* out_y, float* out_lv) {
    if (!c || !x || n <= 0 || !out_y) return fail(VAEB_ERR_ARG, "bad arguments");
    if (out_lv && !gaussian(c)) return fail(VAEB_ERR_ARG, "the log-sigma head exists for the Gaussian decoder only");
    if (out_lv && is_bf16(c)) return fail(VAEB_ERR_ARG, "the log-sigma output is served by fp32 contexts");
    if (n_samples <= 0) return eval_rows(c, x, n, MODE_RECON, out_y, nullptr, out_lv);
    const bool host = c->eps_mode == VAEB_EPS_HOST;
    if (host && c->eps_rows != n * n_samples)
        return fail(VAEB_ERR_STATE, "host eps mode: sampled reconstruct needs eps for %lld rows (n * n_samples), pushed %lld",
                    (long long)(n * n_samples), (long long)c->eps_rows);
    const vaeb_config& g = c->c;
    const int chunk = g.max_eval_rows;
    if (!c->yacc) {
        if (int rc = dalloc(&c->yacc, (size_t)chunk * g.D * (gaussian(c) ? 2 : 1))) return rc;
    }
    float* lacc = gaussian(c) ? c->yacc + (size_t)chunk * g.D : nullptr;
    int epar = c->par;
    if (!is_bf16(c)) if (int rc = eval_arena(c, &epar)) return rc;
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
        const int rows = (int)std::min<int64_t>(chunk, n - r0);
        const int64_t ny = (int64_t)rows * g.D;
        if (is_bf16(c)) {
            if (int rc = bf_upload_rows(c, x + r0 * g.D, rows, c->bf.xeval)) return rc;
        } else {
            HIP_TRY(hipMemcpyAsync(c->xeval, x + r0 * g.D, sizeof(float) * (size_t)ny, hipMemcpyHostToDevice, c->s));
        }
        for (int sidx = 0; sidx < n_samples; ++sidx) {
            const uint32_t domain = 1u | ((uint32_t)(sidx + 1) << 1);
            const float* eps = (host && c->eps_in) ? c->eps_in + ((int64_t)sidx * n + r0) * g.Z : nullptr;
            Prof pr{c, false};
            if (is_bf16(c)) {
                BfFwd f{};
                f.Mb = rows; f.mode = MODE_EVAL; f.train = false; f.x = c->bf.xeval; f.xb = h16c::BatchRef{};
                f.row_base_mul = 0; f.row_base_add = r0;
                f.eps_in = eps; f.eps_in_ld = c->eps_rows; f.domain = domain;
                f.yout = c->y;
                if (int rc = bf_forward(c, c->par, f, pr)) return rc;
            } else {
                StepArgs a = make_args(c, epar, rows, MODE_RECON, c->xeval, false);
                a.L = 1; a.Me = a.Mbp;
                a.eps_mode = host ? 1 : 0;
                a.domain = domain;
                a.row_base_add = r0;
                a.eps_in = eps; a.eps_in_ld = c->eps_rows;
                if (int rc = enqueue_forward(c, a, pr)) return rc;
            }
            const float scale = (sidx == n_samples - 1) ? (float)n_samples : 0.f;
            const dim3 grid((unsigned)std::min<int64_t>(1024, cdiv(ny, 256)));
            hipLaunchKernelGGL(recon_accum_kernel, grid, dim3(256), 0, c->s, c->yacc, c->y, ny, sidx == 0 ? 1 : 0, scale);
            CHECK_LAUNCH();
            if (out_lv) {
                hipLaunchKernelGGL(recon_accum_kernel, grid, dim3(256), 0, c->s, lacc, c->dA6, ny, sidx == 0 ? 1 : 0, scale);
                CHECK_LAUNCH();
            }
        }
        HIP_TRY(hipMemcpyAsync(out_y + r0 * g.D, c->yacc, sizeof(float) * (size_t)ny, hipMemcpyDeviceToHost, c->s));
        if (out_lv)
            HIP_TRY(hipMemcpyAsync(out_lv + r0 * g.D, lacc, sizeof(float) * (size_t)ny, hipMemcpyDeviceToHost, c->s));
        HIP_TRY(hipStreamSynchronize(c->s));
    }
    return 0;
}

// The decoder from a given z (freyFace.py:173-187 `image(z)`, compiled at :237-245; VAEB.py
// :253-265): hd = tanh(z W1 + b1), mu = sigmoid(hd W2 + b2), and for the Gaussian decoder the
// log-sigma head hd W6 + b6 (out_lv).  fp32 contexts; z is [n x Z] row-major.
int vaeb_decode(vaeb_ctx* c, const float* z, int64_t n, float* out_mu, float* out_lv) {
    if (!c || !z || n <= 0 || !out_mu) return fail(VAEB_ERR_ARG, "bad arguments");
    if (out_lv && !gaussian(c)) return fail(VAEB_ERR_ARG, "the log-sigma head exists for the Gaussian decoder only");
    if (is_bf16(c)) return fail(VAEB_ERR_ARG, "vaeb_decode is served by fp32 contexts");
    const vaeb_config& g = c->c;
    const int chunk = g.max_eval_rows;
    int epar = c->par;
    if (int rc = eval_arena(c, &epar)) return rc;
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
        const int rows = (int)std::min<int64_t>(chunk, n - r0);
        StepArgs a = make_args(c, epar, rows, MODE_RECON, c->xeval, false);
        a.L = 1; a.Me = a.Mbp;
        // z rows, pad rows zero (PDecHid writes hd = 0 there)
        HIP_TRY(hipMemsetAsync(c->z, 0, sizeof(float) * (size_t)a.Mbp * g.Z, c->s));
        HIP_TRY(hipMemcpyAsync(c->z, z + r0 * g.Z, sizeof(float) * (size_t)rows * g.Z, hipMemcpyHostToDevice, c->s));
        launch_tile<1, 4, 1, 1, 8>(c->s, PDecHid{a, a.Me, a.H, a.Z});
        CHECK_LAUNCH();
        if (gaussian(c)) launch_bigk<2>(c->s, PDecOut{a, nullptr, a.Me, a.D, a.H});
        else launch_bigk<1>(c->s, PDecOut{a, nullptr, a.Me, a.D, a.H});
        CHECK_LAUNCH();
        HIP_TRY(hipMemcpyAsync(out_mu + r0 * g.D, c->y, sizeof(float) * (size_t)rows * g.D, hipMemcpyDeviceToHost, c->s));
        if (out_lv)
            HIP_TRY(hipMemcpyAsync(out_lv + r0 * g.D, c->dA6, sizeof(float) * (size_t)rows * g.D, hipMemcpyDeviceToHost, c->s));
    }
    HIP_TRY(hipStreamSynchronize(c->s));
    return 0;
}

int vaeb_comm_unique_id(uint8_t out_id[128]) {
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(VAEB_ERR_COMM, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    memcpy(out_id, &id, 128);
    return 0;
}

int vaeb_comm_init(vaeb_ctx* c, const uint8_t id_bytes[128], int32_t rank, int32_t world) {
    if (!c || !id_bytes || world <= 0 || rank < 0 || rank >= world) return fail(VAEB_ERR_ARG, "bad comm arguments");
    if (int rc = w2_flush(c)) return rc;   // a pending deferred dW2 (vaeb_ctx::dw2_defer)
    if ((c->c.estimator == VAEB_EST_FV && world > 1) || c->c.estimator == VAEB_EST_FVS)
        return fail(VAEB_ERR_ARG, "the full-variational paths are single-rank");
    if (c->comm) return fail(VAEB_ERR_STATE, "communicator already initialised");
    HIP_TRY(hipSetDevice(c->c.device));
    // Bucket A's all-reduce + Adagrad on a second stream beside the backward, where the
    // window it can hide behind is longer than what the fork costs.  The graph's fork and
    // join cost ~19 us per step whatever the world size (fp32 MNIST at world 1: 66.0 vs
    // 47.1 us, profiles/r3/dp_world1_start.txt), and on the fp32 engine the backward left
    // after dW2 (| dW6) is the one last launch, ~10 us: at most 10 us of all-reduce could
    // hide there at ANY world size, so the fp32 step never forks.  On the bf16 engine
    // (config 5) the window is ~500 us and bucket A (34 MB) alone is worth the fork at
    // world 1 already (933 vs ~940 us per step), so it always forks.
    c->dp_overlap = is_bf16(c);
    if (const char* ov = getenv("VAEB_DP_OVERLAP")) c->dp_overlap = atoi(ov) != 0;
    // sharded optimizer at world > 1 (dp_reduce_update); VAEB_DP_SHARD=1 forces it at world 1 (tests)
    c->dp_shard = world > 1;
    if (const char* sh = getenv("VAEB_DP_SHARD")) c->dp_shard = atoi(sh) != 0;
    if (!c->s2) {
        HIP_TRY(hipStreamCreateWithFlags(&c->s2, hipStreamNonBlocking));
        for (auto& ev : c->dp_ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    ncclUniqueId id;
    memcpy(&id, id_bytes, 128);
    ncclResult_t r = ncclCommInitRank(&c->comm, world, id, rank);
    if (r != ncclSuccess) return fail(VAEB_ERR_COMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
    c->rank = rank;
    c->world = world;
    free_graphs(c);
    c->graph_failed = false;
    return 0;
}

static const struct { const char* name; int which; } kActs[] = {
    {"h", 0}, {"mu", 1}, {"lv", 2}, {"eps", 3}, {"z", 4}, {"hd", 5}, {"dA2", 6}, {"dA6", 7},
    {"dA1", 8}, {"dZ", 9}, {"dMuLv", 10}, {"dA3", 11}, {"y", 12}, {"kl_part", 13}, {"lp_part", 14}};

int vaeb_get_activation(vaeb_ctx* c, const char* name, float* out, int64_t n) {
    if (!c || !name || !out) return fail(VAEB_ERR_ARG, "null argument");
    float* ptrs[] = {c->h, c->mu, c->lv, c->eps, c->z, c->hd, c->dA2, c->dA6, c->dA1, c->dZ, c->dMuLv, c->dA3, c->y,
                     c->kl_part, c->lp_part};
    if (strcmp(name, "dZ") == 0 && fused_latent(c) && c->fold_bwd && !is_bf16(c) && ho_dz(c) == 1)
        return fail(VAEB_ERR_STATE, "dZ is not stored by the atomic latent hand-off (fan-in <= 16, latent_bwd.hpp): "
                                    "create the context with VAEB_ATOMIC_HO=0 to read it");
    const int64_t R = c->cap, RL = (int64_t)c->cap * c->c.L, D = c->c.D, H = c->c.H, Z = c->c.Z;
    const int64_t cap[] = {R * H, R * Z, R * Z, RL * Z, RL * Z, RL * H, RL * D, RL * D, RL * H, RL * Z, R * 2 * Z,
                           R * H, RL * D, RL * cdiv(Z, 16), RL * cdiv(D, 16)};
    for (auto& a : kActs)
        if (strcmp(a.name, name) == 0) {
            if (!ptrs[a.which]) return fail(VAEB_ERR_STATE, "activation %s not allocated", name);
            if (n < 0 || n > cap[a.which])
                return fail(VAEB_ERR_ARG, "activation %s holds %lld floats, %lld requested", name,
                            (long long)cap[a.which], (long long)n);
            HIP_TRY(hipStreamSynchronize(c->s));
            HIP_TRY(hipMemcpy(out, ptrs[a.which], sizeof(float) * n, hipMemcpyDeviceToHost));
            return 0;
        }
    return fail(VAEB_ERR_ARG, "unknown activation '%s'", name);
}

int vaeb_profile_steps(vaeb_ctx* c, int32_t n_steps, float* out_ms, int32_t* out_ids, int32_t max_k,
                       int32_t* out_nk) {
    if (!c || !out_ms || n_steps <= 0) return fail(VAEB_ERR_ARG, "bad arguments");
    if (int rc = w2_flush(c)) return rc;
    if (!c->data) return fail(VAEB_ERR_STATE, "no data");
    constexpr int kReps = 8;   // each launch issued 8x back to back inside its event bracket
    std::vector<int32_t> order((size_t)n_steps * kReps);
    const int64_t nb = c->nrows / c->c.B_global;
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int32_t)(i % nb);
    if (int rc = upload_order(c, order.data(), (int)order.size())) return rc;
    std::vector<double> tot(kMaxProfKernels, 0.0);
    c->prof_reps = kReps;
    for (int it = 0; it < n_steps; ++it) {
        // 1 ms hold: the eager launches queue up behind it (no host-launch gaps)
        hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, c->s, (uint64_t)100000);
        CHECK_LAUNCH();
        int rc = enqueue_train_step(c, c->par, true);
        if (rc) { c->prof_reps = 1; return rc; }
        if (flips(c)) c->par ^= 1;   // repeats all read arena par and write par ^ 1
        HIP_TRY(hipStreamSynchronize(c->s));
        for (int k = 0; k + 1 < c->prof_n; ++k) {
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, c->pev[k], c->pev[k + 1]));
            tot[k] += ms / kReps;
        }
    }
    c->prof_reps = 1;
    const int nk = std::max(0, c->prof_n - 1);
    for (int k = 0; k < nk && k < max_k; ++k) {
        out_ms[k] = (float)(tot[k] / n_steps);
        if (out_ids) out_ids[k] = c->prof_ids[k];
    }
    if (out_nk) *out_nk = nk;
    return 0;
}

int vaeb_debug_timeline(vaeb_ctx* c, int32_t batch_index, uint64_t* out, int64_t cap, int32_t* out_launches) {
    if (!c || !out) return fail(VAEB_ERR_ARG, "bad arguments");
    if (int rc = w2_flush(c)) return rc;
    if (int rc = check_batches(c, &batch_index, 1)) return rc;
    const size_t n = (size_t)kMaxProfKernels * kDbgWG * 8;
    if (!c->dbg)
        if (int rc = dalloc(&c->dbg, n)) return rc;
    HIP_TRY(hipMemsetAsync(c->dbg, 0, n * sizeof(uint64_t), c->s));
    if (int rc = upload_order(c, &batch_index, 1)) return rc;
    c->dbg_slot = 0;
    int rc = enqueue_train_step(c, c->par, false);
    if (flips(c)) c->par ^= 1;
    const int launches = c->dbg_slot;
    c->dbg_slot = 0;
    uint64_t* d = c->dbg;
    c->dbg = nullptr;  // later steps (and captured graphs) run without stamps
    if (rc) { hipFree(d); return rc; }
    HIP_TRY(hipStreamSynchronize(c->s));
    const size_t m = std::min<size_t>(n, (size_t)cap);
    HIP_TRY(hipMemcpy(out, d, m * sizeof(uint64_t), hipMemcpyDeviceToHost));
    hipFree(d);
    if (out_launches) *out_launches = launches;
    return 0;
}

int vaeb_test_gemm_bf16(vaeb_ctx* c, int32_t ako, int32_t bko, int32_t M, int32_t N, int32_t K, const float* A,
                        const float* B, float* C, int32_t ksplit) {
    if (!c) return fail(VAEB_ERR_ARG, "null ctx");
    return is_f16(c) ? eng_hf::h16_test_gemm(c, ako, bko, M, N, K, A, B, C, ksplit)
                     : eng_bf::h16_test_gemm(c, ako, bko, M, N, K, A, B, C, ksplit);
}

int vaeb_bench_gemm_bf16(vaeb_ctx* c, int32_t ako, int32_t bko, int32_t M, int32_t N, int32_t K, int32_t bn,
                         int32_t reps, float* out_ms) {
    if (!c) return fail(VAEB_ERR_ARG, "null ctx");
    return is_f16(c) ? eng_hf::h16_bench_gemm(c, ako, bko, M, N, K, bn, reps, out_ms)
                     : eng_bf::h16_bench_gemm(c, ako, bko, M, N, K, bn, reps, out_ms);
}

int vaeb_time_update_many(vaeb_ctx* c, const int32_t* idx, int32_t n, float* out_gpu_ms, double* out_enqueue_ms) {
    if (!c || !out_gpu_ms) return fail(VAEB_ERR_ARG, "null argument");
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipStreamSynchronize(c->s));
    HIP_TRY(hipEventRecord(e0, c->s));
    const auto t0 = std::chrono::steady_clock::now();
    int rc = vaeb_update_many(c, idx, n);
    const auto t1 = std::chrono::steady_clock::now();
    if (rc == 0) {
        hipEventRecord(e1, c->s);
        hipEventSynchronize(e1);
        hipEventElapsedTime(out_gpu_ms, e0, e1);
        if (out_enqueue_ms) *out_enqueue_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return rc;
}

int vaeb_busy(vaeb_ctx* c, int32_t us) {
    if (!c || us <= 0) return fail(VAEB_ERR_ARG, "bad arguments");
    hipLaunchKernelGGL(busy_kernel, dim3(2048), dim3(256), 0, c->s, (uint64_t)us * 100, c->fv_part);
    CHECK_LAUNCH();
    return 0;
}

int vaeb_graph_status(vaeb_ctx* c, int32_t* mode, char* msg, int32_t cap) {
    if (!c || !mode) return fail(VAEB_ERR_ARG, "null argument");
    if (!c->c.use_graph) *mode = VAEB_GRAPH_OFF;
    else if (c->graph_failed) *mode = VAEB_GRAPH_EAGER_FALLBACK;
    else *mode = c->gN[0][1] ? VAEB_GRAPH_REPLAY : VAEB_GRAPH_NOT_CAPTURED;
    if (msg && cap > 0) snprintf(msg, (size_t)cap, "%s", c->graph_failed ? c->graph_err.c_str() : "");
    return 0;
}

int vaeb_comm_info(vaeb_ctx* c, int32_t* rccl_version, int32_t* dp_overlap, int32_t* world) {
    if (!c) return fail(VAEB_ERR_ARG, "null ctx");
    if (rccl_version) {
        int v = 0;
        ncclResult_t r = ncclGetVersion(&v);
        if (r != ncclSuccess) return fail(VAEB_ERR_COMM, "ncclGetVersion: %s", ncclGetErrorString(r));
        *rccl_version = v;
    }
    if (dp_overlap) *dp_overlap = c->comm ? (c->dp_overlap ? 1 : 0) : -1;
    if (world) *world = c->comm ? c->world : 1;
    return 0;
}

int vaeb_dp_plan(const vaeb_config* cfg, int32_t world, int32_t rank, int32_t sharded, int32_t bucket,
                 int64_t* out_P, int64_t* runs, int32_t* out_nrun, int64_t* own, int32_t* out_nown, int32_t* out_book,
                 int64_t* foreign, int32_t* out_nforeign) {
    if (!cfg || world <= 0 || rank < 0 || rank >= world || bucket < 0 || bucket > 2)
        return fail(VAEB_ERR_ARG, "bad plan arguments");
    if (cfg->D <= 0 || cfg->H <= 0 || cfg->Z <= 0) return fail(VAEB_ERR_ARG, "dimensions must be positive");
    // a host-only context holding exactly the fields the plan functions read (no stream, no
    // allocation): the same code dp_reduce_update runs on a rank
    vaeb_ctx c;
    c.c = *cfg;
    set_arena_layout(&c);
    c.world = world;
    c.rank = rank;
    c.dp_shard = sharded != 0;
    const DpBucket bk = bucket == 0 ? dp_bucket_a_runs(&c) : bucket == 1 ? dp_bucket_b_runs(&c) : dp_bucket_all_runs(&c);
    if (out_P) *out_P = c.P;
    if (runs)
        for (int j = 0; j < bk.nrun; ++j) {
            runs[3 * j] = bk.lo[j];
            runs[3 * j + 1] = bk.n[j];
            runs[3 * j + 2] = dp_shard_len(&c, bk.n[j]);
        }
    if (out_nrun) *out_nrun = bk.nrun;
    auto put = [](const DpRange& r, int64_t* dst, int32_t* cnt) {
        int k = 0;
        while (k < kDpRuns && r.n[k]) {
            if (dst) { dst[2 * k] = r.lo[k]; dst[2 * k + 1] = r.n[k]; }
            ++k;
        }
        if (cnt) *cnt = k;
    };
    const DpRange o = dp_opt_range(&c, bk);
    put(o, own, out_nown);
    if (out_book) *out_book = o.book;
    put(dp_foreign_range(&c, bk), foreign, out_nforeign);
    return 0;
}

}  // extern "C"

// vaeb_dp_rank_update's body, with the context's (world, rank, dp_shard) already set to the
// emulated rank's: the reduce-scatter's result uploaded, this rank's optimizer launch, the
// all-gather's result uploaded, the bf16 shadow fix -- dp_reduce_update with its collectives
// replaced by host copies, the kernels and index ranges unchanged.
static int dp_rank_update_body(vaeb_ctx* c, int bucket, const float* gsum, const float* thg) {
    const int par = c->par;
    hipStream_t s = c->s;
    const bool bf = is_bf16(c);
    const DpBucket bk = bucket == 0 ? dp_bucket_a_runs(c) : bucket == 1 ? dp_bucket_b_runs(c) : dp_bucket_all_runs(c);
    DpRange own = dp_opt_range(c, bk);
    own.book = 0;   // the SGVB bookkeeping (value, epoch sums, cursor, step) is not emulated
    const DpRange fr = dp_foreign_range(c, bk);
    // a step's first bucket (A, or all): the out arena -- theta' and the bf16 shadow -- NaN first,
    // so every element the step leaves there was written by it
    if (bucket != 1) {
        HIP_TRY(hipMemsetAsync(c->theta2[par ^ 1], 0xff, sizeof(float) * (size_t)c->P, s));
        if (bf) HIP_TRY(hipMemsetAsync(c->bf.shadow2[par ^ 1], 0xff, sizeof(bf16_t) * (size_t)c->bf.S, s));
    }
    // the reduce-scatter (+ all-reduce of the remainders): this rank's destinations hold the sum;
    // every other gradient element is NaN (the optimizer must not read it)
    HIP_TRY(hipMemsetAsync(c->grad, 0xff, sizeof(float) * (size_t)(c->P + 1), s));
    for (int k = 0; k < kDpRuns; ++k)
        if (own.n[k])
            HIP_TRY(hipMemcpyAsync(c->grad + own.lo[k], gsum + own.lo[k], sizeof(float) * (size_t)own.n[k],
                                   hipMemcpyHostToDevice, s));
    if (int rc = bf ? h16_dp_opt(c, par, own) : dp_opt_launch(c, s, make_opt(c, par, true, false), own, ElboArgs{}))
        return rc;
    if (thg) {
        // the all-gather: the other ranks' theta' shards into the out arena, then their shadow
        for (int k = 0; k < kDpRuns; ++k)
            if (fr.n[k])
                HIP_TRY(hipMemcpyAsync(c->theta2[par ^ 1] + fr.lo[k], thg + fr.lo[k], sizeof(float) * (size_t)fr.n[k],
                                       hipMemcpyHostToDevice, s));
        if (bf) if (int rc = h16_dp_fix(c, par, fr)) return rc;
    }
    HIP_TRY(hipStreamSynchronize(s));
    return 0;
}

extern "C" {

int vaeb_dp_rank_update(vaeb_ctx* c, int32_t world, int32_t rank, int32_t bucket, const float* grad_sum,
                        int64_t n_grad, const float* theta_gathered, int32_t finish) {
    if (!c || !grad_sum || world <= 0 || world > 64 || rank < 0 || rank >= world || bucket < 0 || bucket > 2)
        return fail(VAEB_ERR_ARG, "bad dp_rank_update arguments");
    if (c->comm) return fail(VAEB_ERR_STATE, "vaeb_dp_rank_update emulates the collectives: use a context without a communicator");
    if (c->c.estimator == VAEB_EST_FV || c->c.estimator == VAEB_EST_FVS)
        return fail(VAEB_ERR_STATE, "the FV estimators have no data-parallel optimizer");
    if (n_grad != c->P + 1) return fail(VAEB_ERR_ARG, "size mismatch: got %lld, expected %lld", (long long)n_grad, (long long)(c->P + 1));
    if (int rc = w2_flush(c)) return rc;
    HIP_TRY(hipStreamSynchronize(c->s));
    const int w0 = c->world, r0 = c->rank;
    const bool s0 = c->dp_shard;
    c->world = world; c->rank = rank; c->dp_shard = world > 1;
    const int rc = dp_rank_update_body(c, bucket, grad_sum, theta_gathered);
    c->world = w0; c->rank = r0; c->dp_shard = s0;
    if (rc) return rc;
    if (finish) c->par ^= 1;
    return 0;
}

int vaeb_get_shadow(vaeb_ctx* c, uint16_t* out, int64_t n) {
    if (!c || !out) return fail(VAEB_ERR_ARG, "null argument");
    if (!is_bf16(c)) return fail(VAEB_ERR_STATE, "only the bf16 engine keeps a shadow arena");
    const int64_t nw = c->bf.smap.nweights;
    if (n != nw) return fail(VAEB_ERR_ARG, "size mismatch: got %lld, expected %lld", (long long)n, (long long)nw);
    if (int rc = w2_flush(c)) return rc;
    bf16_t* tmp = nullptr;
    if (int rc = dalloc(&tmp, (size_t)nw)) return rc;
    hipLaunchKernelGGL(bf::shadow_gather_kernel, dim3(1024), dim3(256), 0, c->s, (const bf16_t*)c->bf.shadow2[c->par], tmp,
                       c->bf.smap);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->s);
    if (e == hipSuccess) e = hipMemcpy(out, tmp, sizeof(bf16_t) * (size_t)nw, hipMemcpyDeviceToHost);
    hipFree(tmp);
    if (e != hipSuccess) return fail(VAEB_ERR_HIP, "vaeb_get_shadow: %s", hipGetErrorString(e));
    return 0;
}

int vaeb_kernel_name(int32_t id, char* out, int32_t cap) {
    if (!out || cap <= 0) return fail(VAEB_ERR_ARG, "bad buffer");
    const int n = (int)(sizeof(kKernelNames) / sizeof(kKernelNames[0]));
    if (id < 0 || id >= n) return fail(VAEB_ERR_ARG, "unknown kernel id %d", id);
    snprintf(out, (size_t)cap, "%s", kKernelNames[id]);
    return 0;
}

}  // extern "C"

// degenerate-vae autoencoder (vaeb_ae_*) on the same fp32 tile engine
#include "engine_ae.inc"
