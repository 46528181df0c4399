#!/usr/bin/env python3
"""Benchmark: SGVB training images/sec + ELBO at MNIST 784-500-20, batch 100 per GPU.

A "step" is one VAEB.update (/root/reference/VAEB.py:408-415) on one minibatch of
synthetic rows: encoder -> reparameterised sample -> decoder -> ELBO + KL -> gradient ->
Adagrad, all on the GPU (libvaeb_hip.so); the training set is resident in HBM before
timing starts.  With N GPUs every rank processes its own B rows of a B*N-row global
minibatch and the gradients are all-reduced over RCCL ("weak" scaling).

Configs (BASELINE.json):
  --config mnist (default, the headline metric): 784-500-20 Bernoulli, B=100, fp32 MFMA
  --config frey  (Frey-shaped, BASELINE config 1 shapes): 560-200-2 Gaussian decoder, B=100, fp32
  --config fv    (config 4): literal --full_varational step, MNIST 784-500-20, B=100, fp32
  --config fvs   (config 4, weight-posterior reparam extension): FV with theta~ = mu + |sigma| zeta
  --config synth (config 5, roofline stress): 4096-2048-128 Bernoulli, B=8192 per GPU,
                 fp16 MFMA operands (--dtype bf16: bf16) / fp32 accumulation and master weights

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--config mnist|frey|fv|fvs|synth]
                       [--scaling weak|strong]
        (N > 1: torch.distributed.run, one process per GPU)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

PEAK_F32_TFLOPS = 157.3    # MI355X f32 MFMA / vector peak (MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 / fp16 MFMA peak (no sparsity; the same rate for both)
PEAK_HBM_GBS = 8000.0


def phase_flops(D, H, Z, B, L=1, gaussian=False):
    """Algorithmic FLOPs per launch of each kernel (2 per multiply-add)."""
    g = 2 if gaussian else 1
    return {
        "p1_enc": 2 * B * D * H,
        "p2_heads": 2 * B * H * 2 * Z,
        "p3_dechid": 2 * L * B * Z * H,
        "p4_decout": 2 * L * B * H * D * g,
        "p5_dhd": 2 * L * B * D * H * g,
        "p6_dz": 2 * L * B * H * Z,
        "p7_dh": 2 * B * 2 * Z * H,
        "p8_wgrad_w2": 2 * L * B * H * D * g,
        "p8_wgrad_w1": 2 * L * B * Z * H,
        "p8_wgrad_w3w45": 2 * B * (D * H + H * 2 * Z),
        "p23_heads_dechid": 2 * B * H * 2 * Z + 2 * L * B * Z * H,
        # horizontally fused launches (hfuse.hpp): phase + weight-gradient tiles in one grid
        "p5_dhd_w2": 2 * L * B * D * H * g + 2 * L * B * H * D * g,
        "p67_dz_dh_w1": 2 * L * B * H * Z + 2 * B * 2 * Z * H + 2 * L * B * Z * H,
        # folded latent block (latent.hpp): encoder GEMM + heads; hd recompute + decoder GEMM
        "p1_enc_latent": 2 * B * D * H + 2 * B * H * 2 * Z,
        "p4_decout_z": 2 * L * B * Z * H + 2 * L * B * H * D * g,
        # bf16 engine (step_bf16.hpp)
        "bf_enc": 2 * B * D * H,
        "bf_heads": 2 * B * H * 2 * Z,
        "bf_dechid": 2 * L * B * Z * H,
        "bf_decout": 2 * L * B * H * D * g,
        "bf_dhd": 2 * L * B * D * g * H,
        "bf_dW26": 2 * L * B * H * D * g,
        "bf_dz": 2 * L * B * H * Z,
        "bf_dW1": 2 * L * B * Z * H,
        "bf_dh": 2 * B * 2 * Z * H,
        "bf_dW45": 2 * B * H * 2 * Z,
        "bf_dW3": 2 * B * D * H,
        "bf_dhd_dW26": 2 * L * B * D * g * H + 2 * L * B * H * D * g,   # one grid (gemm2_kernel)
        # folded latent backward (latent_bwd.hpp): dhd + dZ slabs + latent backward | dW2; the
        # last launch dW3 (dA3 formed in-workgroup) | dW45 | dW1
        "p5_dhd_dz_w2": 2 * L * B * D * H * g + 2 * L * B * H * Z + 2 * L * B * H * D * g,
        "p8_wgrad_w3w45w1": 2 * B * (D * H + H * 2 * Z) + 2 * B * 2 * Z * H + 2 * L * B * Z * H,
        # deferred dW2 (round 4): the encoder launch also runs the previous step's dW2 tiles,
        # the dhd launch has none
        "p1_enc_latent_w2": 2 * B * D * H + 2 * B * H * 2 * Z + 2 * L * B * H * D * g,
        "p5_dhd_dz": 2 * L * B * D * H * g + 2 * L * B * H * Z,
    }


def step_flops(D, H, Z, B, L=1, gaussian=False):
    """2B(2DH + 9HZ + 3HD) (Bernoulli, L=1)."""
    g = 2 if gaussian else 1
    return 2 * B * (D * H + 2 * H * Z) + 2 * L * B * (Z * H + g * H * D) + \
        2 * L * B * (g * D * H + H * Z + Z * H + g * H * D) + 2 * B * (2 * Z * H + H * 2 * Z + D * H)


KERNEL_SYMBOLS = {"p1_enc": "PEnc", "p23_heads_dechid": "heads_dechid_kernel", "p4_decout": "PDecOut",
                  "p5_dhd_w2": "vaeb::tile_wgrad_kernel", "p67_dz_dh_w1": "vaeb::dz_dh_wgrad_kernel",
                  "fv_update": "vaeb::fv_kernel", "fvs_update": "vaeb::fvs_update_kernel",
                  "fvs_sample": "vaeb::fvs_sample_kernel",
                  "p8_wgrad_w3w45": "vaeb::wgrad_kernel",
                  "p1_enc_latent": ("vaeb::enc_latent",),   # enc_latent_kernel | enc_latent_fv_kernel
                  "p4_decout_z": ("vaeb::decout_z",),   # decout_z_kernel | decout_z2_kernel
                  # bf16 GEMMs are one template: the epilogue / layout pair names the launch (all
                  # substrings of a tuple must appear; a list holds alternatives, the current form
                  # first: the 8-phase 256 x 256 loop, then the ring forms of earlier rounds)
                  "bf_enc": [("gemm8_kernel<0, 1,", "EpiBiasAct>"), ("gemm_kernel<0, 1, 256,", "EpiBiasAct")],
                  "bf_dechid": [("gemm_kernel<0, 1, 128,", "EpiBiasAct"), ("gemm8_kernel<0, 1,", "EpiBiasAct>")],
                  "bf_heads": [("EpiHeadsLatent",)], "bf_dz": [("EpiDzLatent",)],
                  "bf_decout": [("EpiDecOutT>",), ("EpiDecOut<false>",)],
                  "bf_dh": [("gemm8_kernel<0, 0,", "EpiDTanhT>"), ("gemm_kernel<0, 0,", "EpiDTanh>")],
                  "bf_dhd": [("EpiDTanhTDz>",), ("gemm8_kernel<0, 0,", "EpiDTanhT>"), ("gemm_kernel<0, 0,", "EpiDTanh>")],
                  "bf_dW26": ("EpiAdagrad",),
                  "bf_dW3": [("gemm8_kernel<1, 1,", "EpiAdagrad>"), ("gemm_kernel<1, 1,", "EpiAdagrad,")],
                  "bf_dhd_dW26": ("2_kernel<1, 1,",),   # gemm2_kernel | gemm8x2_kernel
                  "p5_dhd_dz_w2": "vaeb::dhd_dz_wgrad_kernel", "p8_wgrad_w3w45w1": "vaeb::wgrad3_kernel",
                  "p1_enc_latent_w2": ("vaeb::enc_latent16_w2",), "p5_dhd_dz": "vaeb::dhd_dz_wgrad_kernel"}
PMC_ROUNDS = ("r6", "r5", "r4")   # the newest round whose committed PMC passes give roofline.traffic (traffic_source)
PMC_FILES = {c: next((p for p in (os.path.join(ROOT, "profiles", r, f"pmc_{c}_per_launch.json") for r in PMC_ROUNDS)
                      if os.path.exists(p)), os.path.join(ROOT, "profiles", PMC_ROUNDS[-1], f"pmc_{c}_per_launch.json"))
             for c in ("mnist", "frey", "fv", "fvs", "synth")}


def committed_traffic(kernel, path=PMC_FILES["mnist"], symbols=KERNEL_SYMBOLS):
    """HBM bytes per launch of `kernel` from the rocprofv3 PMC passes committed under
    profiles/ (separate FETCH_SIZE / WRITE_SIZE passes folded by scripts/pmc_summary.py,
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM).  Kernels whose symbol
    is shared by several launches of a step report the per-launch average of all of them."""
    try:
        data = json.load(open(path))
    except Exception:
        return None
    sym = symbols.get(kernel)
    if not sym:
        return None
    alts = sym if isinstance(sym, list) else [(sym,) if isinstance(sym, str) else sym]
    for alt in alts:
        for name, v in data.items():
            if all(t in name for t in alt) and "hbm_bytes_per_launch" in v:
                return v["hbm_bytes_per_launch"]
    return None


def host_cpu_info():
    """(threads to use, nproc, CPU model).  The GPU box shares its host among the GPUs and
    pins OMP_NUM_THREADS to this job's share (16 per GPU): os.cpu_count() reports the
    whole machine, so the baseline uses the share (OMP_NUM_THREADS, else the affinity
    mask) and records nproc beside it."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:  # pragma: no cover
        aff = nproc
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(aff, share) if share > 0 else aff)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:  # pragma: no cover
        pass
    return threads, nproc, model


def _threads_ctx(n):
    try:
        from threadpoolctl import threadpool_limits
        return threadpool_limits(limits=n)
    except Exception:  # pragma: no cover
        return None


def cpu_baseline_pair(fn, budget_s, single_kw=None, **kw):
    """Time `fn` (a bounded oracle run returning (steps, seconds, images)) on the job's host
    thread share, then single-threaded on a shorter budget; one cpu_baseline object."""
    threads, nproc, model = host_cpu_info()
    ctx = _threads_ctx(threads)
    try:
        n, dt, imgs, what = fn(budget_s, **kw)
    finally:
        if ctx is not None and hasattr(ctx, "unregister"):
            ctx.unregister()
    ctx1 = _threads_ctx(1)
    try:
        n1, dt1, imgs1, _ = fn(max(2.0, budget_s / 2), **{**kw, **(single_kw or {})})
    finally:
        if ctx1 is not None and hasattr(ctx1, "unregister"):
            ctx1.unregister()
    multi, single = imgs / dt, imgs1 / dt1
    # the faster of the two is the baseline (at B = 100 the threaded BLAS can lose to one
    # thread); both figures are kept
    best_threads, best = (threads, multi) if multi >= single else (1, single)
    return {"value": best, "unit": "images/s", "cores": best_threads, "kind": "port",
            "threaded_value": multi, "threads": threads, "single_thread_value": single,
            "nproc": nproc, "cpu_model": model,
            "sample": f"{n} {what} in {dt:.1f} s on {threads} OpenBLAS threads (job share of {nproc} CPUs, {model}); "
                      f"1 thread: {n1} steps in {dt1:.1f} s; value = the faster"}


def cpu_baseline(D, H, Z, B, x, budget_s=10.0, max_steps=20000, continuous=False, warm=3, single_kw=None):
    """The oracle's float32 NumPy restatement of the same step, on the host cores."""
    return cpu_baseline_pair(_cpu_run_lb, budget_s, single_kw=single_kw, D=D, H=H, Z=Z, B=B, x=x,
                             max_steps=max_steps, continuous=continuous, warm=warm)


def _cpu_run_lb(budget_s, D, H, Z, B, x, max_steps=20000, continuous=False, warm=3):
    from oracle import vaeb_oracle as O
    cfg = O.Config(D=D, H=H, Z=Z, continuous=continuous)
    params = O.init_params(cfg)
    acc = [np.zeros_like(p) for p in params]
    rng = np.random.default_rng(0)
    nb = x.shape[0] // B
    for i in range(min(warm, max_steps, nb)):  # warm-up
        eps = rng.standard_normal((1, B, Z)).astype(np.float32)
        _, params, acc, _ = O.step(params, acc, x[i * B:(i + 1) * B], eps, cfg)
    n = 0
    t0 = time.perf_counter()
    while True:
        b = n % nb
        eps = rng.standard_normal((1, B, Z)).astype(np.float32)
        _, params, acc, _ = O.step(params, acc, x[b * B:(b + 1) * B], eps, cfg)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= budget_s or n >= max_steps:
            break
    return n, dt, n * B, f"float32 NumPy oracle steps ({D}-{H}-{Z}, B={B})"


def cpu_baseline_fv(D, H, Z, B, x, budget_s=10.0, max_steps=20000, sample=False):
    """The oracle's full-variational step (literal, or with the weight sample: FVS) in
    float32 NumPy on the host cores."""
    return cpu_baseline_pair(_cpu_run_fv, budget_s, D=D, H=H, Z=Z, B=B, x=x, max_steps=max_steps, sample=sample)


def _cpu_run_fv(budget_s, D, H, Z, B, x, max_steps=20000, sample=False):
    from oracle import vaeb_oracle as O
    cfg = O.Config(D=D, H=H, Z=Z, estimator="FV")
    theta = O.init_params(cfg)
    mu = [t.copy() for t in theta]
    sig = [np.full_like(t, 1e-3) for t in theta]
    am = [np.zeros_like(t) for t in theta]
    as_ = [np.zeros_like(t) for t in theta]
    rng = np.random.default_rng(0)
    nb = x.shape[0] // B
    n, t0 = 0, time.perf_counter()
    while True:
        b = n % nb
        eps = rng.standard_normal((1, B, Z)).astype(np.float32)
        if sample:
            zeta = [rng.standard_normal(t.shape).astype(np.float32) for t in theta]
            _, mu, sig, am, as_, _ = O.fvs_step(mu, sig, am, as_, x[b * B:(b + 1) * B], eps, zeta, cfg)
        else:
            _, mu, sig, am, as_, _ = O.fv_step(theta, mu, sig, am, as_, x[b * B:(b + 1) * B], eps, cfg)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= budget_s or n >= max_steps:
            break
    return n, dt, n * B, f"float32 NumPy oracle {'FVS' if sample else 'FV'} steps ({D}-{H}-{Z}, B={B})"


CONFIGS = {
    "mnist": dict(D=784, H=500, Z=20, B=100, N=50000, dtype="f32", steps=2000, warmup=200,
                  metric="SGVB training images/sec + ELBO at MNIST 784-500-20, batch 100",
                  workload="MNIST 784-500-20 Bernoulli decoder, LB estimator, L=1, Adagrad lr 0.01"),
    "frey": dict(D=560, H=200, Z=2, B=100, N=1500, dtype="f32", steps=2000, warmup=200, continuous=True,
                 metric="SGVB training images/sec + ELBO at Frey-shaped 560-200-2 (Gaussian decoder), batch 100",
                 workload="Frey-shaped 560-200-2 Gaussian decoder, LB estimator, L=1, Adagrad lr 0.01 "
                          "(BASELINE config 1 shapes)"),
    "fv": dict(D=784, H=500, Z=20, B=100, N=50000, dtype="f32", steps=2000, warmup=200, estimator="FV",
               metric="Literal full-variational (--full_varational) SGVB step images/sec, MNIST 784-500-20, batch 100",
               workload="MNIST 784-500-20 Bernoulli decoder, FV estimator (fixed theta, Adagrad on mu_theta / "
                        "sigma_theta, sigma 1e-3), L=1, lr 0.01 (BASELINE config 4)"),
    "fvs": dict(D=784, H=500, Z=20, B=100, N=50000, dtype="f32", steps=2000, warmup=200, estimator="FVS",
                metric="Full-variational SGVB step with the weight-posterior sample theta~ = mu + |sigma| zeta, "
                       "images/sec, MNIST 784-500-20, batch 100",
                workload="MNIST 784-500-20 Bernoulli decoder, FVS estimator (extension: weights sampled from "
                         "N(mu, sigma^2) each step, VAEB.py:127-129; Adagrad on mu / sigma), L=1, lr 0.01 "
                         "(BASELINE config 4's weight-posterior reparam)"),
    # BASELINE config 5 names fp16 MFMA: fp16 operands by default (--dtype bf16: the bf16 instantiation)
    "synth": dict(D=4096, H=2048, Z=128, B=8192, N=16 * 8192, dtype="fp16", steps=50, warmup=5,
                  metric="SGVB training images/sec, synthetic 4096-2048-128, batch 8192 per GPU, fp16 MFMA",
                  workload="synthetic 4096-2048-128 Bernoulli decoder, LB, L=1, Adagrad lr 0.01, fp16 operands / "
                           "fp32 accumulate + fp32 master weights (BASELINE config 5)"),
}


def spawn_ranks(n, argv, poll_s=0.2, script=None):
    """`bench.py --gpus N` without a launcher: N rank processes of this script (vaeb_amd.dp)."""
    from vaeb_amd.dp import spawn_ranks as _spawn
    return _spawn(n, [sys.executable, script or os.path.abspath(__file__)] + list(argv), poll_s=poll_s)


DTYPES = {"f32": 0, "bf16": 1, "fp16": 2}   # vaeb_dtype (include/vaeb_hip.h)


def make_context(C, D, H, Z, B, Bg, row_off, local, args, gauss, bf16, dist, rank, world):
    """One library context (and, with world > 1, its RCCL communicator; the 128-byte id
    travels over the gloo group)."""
    from vaeb_amd import _lib
    ctx = _lib.Context(D, H, Z, B, B_global=Bg, row_offset=row_off, device=local,
                       decoder=_lib.DEC_GAUSSIAN if gauss else _lib.DEC_BERNOULLI,
                       estimator={"FV": _lib.EST_FV, "FVS": _lib.EST_FVS}.get(C.get("estimator"), _lib.EST_LB),
                       use_graph=not args.no_graph, max_eval_rows=B if bf16 else 1000,
                       dtype=DTYPES[C["dtype"]])
    if world > 1:
        from vaeb_amd.dp import comm_setup
        comm_setup(ctx, dist, rank, world)
        if world != args.gpus:
            raise SystemExit(f"rank {rank}: the RCCL communicator holds {world} ranks, expected {args.gpus}")
    return ctx


def graph_check(ctx, dist, world):
    """How every rank's steps run (vaeb_graph_status), gathered to all ranks.  With world > 1
    a rank whose graph capture fell back to eager launches ends the run on EVERY rank with a
    non-zero exit: an eager multi-rank step is not the configuration that was tested (the
    library itself also refuses that fallback at world > 1; this covers any other path)."""
    st = list(ctx.graph_status())
    allst = [st]
    if dist:
        allst = [None] * world
        dist.all_gather_object(allst, st)
    bad = [(r, m) for r, (mode, m) in enumerate(allst) if mode == "eager_fallback"]
    if bad and world > 1:
        raise SystemExit(f"graph capture fell back to eager launches on rank(s) {[r for r, _ in bad]}: {bad[0][1]}")
    return [mode for mode, _ in allst]


def timed_run(ctx, order, warmup, steps, dist, world=1, sync=False, warm_ms=0.0):
    """W untimed steps, then exactly K steps between barrier + stream sync; max over ranks.
    sync: the K steps as K synchronous update(index) calls (the reference's loop) instead of
    one update_many.  Returns (seconds, the graph mode of each rank after the warmup)."""
    warm_order, timed_order = order(warmup), order(steps)   # host work done before the GPU runs
    if warm_ms > 0:
        # graph capture first (host-bound: the first call of a context), then the device warm-up
        # kernel, then the W warmup steps proper (the first of which is that captured call)
        if not sync:
            ctx.update_many(warm_order[:1])
            ctx.synchronize()
            ctx.epoch_elbo()
            warm_order = warm_order[1:]
        ctx.busy(int(warm_ms * 1000))
    if sync:
        for b in warm_order:
            ctx.update(int(b))
    else:
        ctx.update_many(warm_order)
    ctx.synchronize()
    ctx.epoch_elbo()
    modes = graph_check(ctx, dist, world)
    if dist:
        dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    if sync:
        for b in timed_order.tolist():
            ctx.update(b)
    else:
        ctx.update_many(timed_order)
    ctx.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    el = t1 - t0
    if dist:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, modes


def comm_record(ctx, dist, world):
    """Per rank: the RCCL version, the overlap choice and the collective algorithm / protocol
    requested through the environment (RCCL picks per call when unset: "auto")."""
    info = dict(ctx.comm_info())
    info["algo"] = os.environ.get("NCCL_ALGO", "auto")
    info["proto"] = os.environ.get("NCCL_PROTO", "auto")
    if not dist:
        return [info]
    out = [None] * world
    dist.all_gather_object(out, info)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="mnist")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-strong", action="store_true", help="N > 1, weak scaling: skip the strong-scaling leg")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--device-warm-ms", type=float, default=30.0,
                    help="before the W warmup steps, keep every CU busy this long (no model state is "
                         "touched): the context's first call captures its graphs on the host (~10 ms, GPU "
                         "idle), and a 20-step timed region right after runs partly below boost clock "
                         "(DESIGN.md 6; 0 disables)")
    ap.add_argument("--sync", action="store_true",
                    help="time the reference's per-step synchronous form: K calls of update(index), each "
                         "returning its SGVB/B (VAEB.py:577-579), instead of one K-step update_many")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: B rows per GPU (default); strong: one B-row global minibatch split "
                         "contiguously over the ranks (100 over 8 = 13,13,13,13,12,12,12,12; SURVEY 8(e))")
    ap.add_argument("--dtype", choices=sorted(DTYPES), default=None,
                    help="operand type (default: the config's; synth: fp16).  fp16 runs config 5 on "
                         "v_mfma_f32_16x16x32_f16 as BASELINE.json names it (DESIGN.md 4.2)")
    argv = sys.argv[1:] if argv is None else list(argv)
    args = ap.parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: one process per GPU, started here before any GPU call
        sys.exit(spawn_ranks(args.gpus, argv))
    C = CONFIGS[args.config]
    if args.dtype and args.dtype != C["dtype"]:
        C = dict(C, dtype=args.dtype)
        for k in ("metric", "workload"):
            C[k] = C[k].replace(CONFIGS[args.config]["dtype"], args.dtype)
    steps = args.steps if args.steps is not None else C["steps"]
    warmup = args.warmup if args.warmup is not None else C["warmup"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}")
    dist = None
    if world > 1:
        import torch.distributed as dist  # host-side coordination only (gloo); the data path is RCCL
        dist.init_process_group("gloo")

    from vaeb_amd.dp import row_split
    from vaeb_amd.model import initial_params
    from vaeb_amd.synthetic import frey_like, mnist_like, synth_like

    D, H, Z = C["D"], C["H"], C["Z"]
    Bn = args.batch if args.batch is not None else C["B"]
    B, row_off, Bg = row_split(Bn, world, rank, args.scaling)
    N = max(C["N"], 4 * Bg)
    bf16 = C["dtype"] in ("bf16", "fp16")   # the 16-bit engine
    gauss = C.get("continuous", False)
    if bf16:
        x = synth_like(N, D=D)             # synth x ~ Bernoulli(0.5)
    elif gauss:
        x = frey_like(n=N, D=D)            # Frey-shaped x ~ Beta(2, 2)
    else:
        x = mnist_like(n=N, D=D)
    fv = C.get("estimator") in ("FV", "FVS")
    if fv and world > 1:
        raise SystemExit("the full-variational paths are single-rank (vaeb_comm_init rejects them)")
    ctx = make_context(C, D, H, Z, B, Bg, row_off, local, args, gauss, bf16, dist, rank, world)
    n_gpus = ctx.comm_count()
    ctx.set_data(x)
    theta0 = np.concatenate([a.ravel() for a in initial_params(D, H, Z, gauss)])
    ctx.set_params(theta0)
    if fv:   # VAEB.py:120-125: mu_theta = theta, sigma_theta = 1e-3, Adagrad state 0
        ctx.set_fv_state(theta0, np.full_like(theta0, 1e-3), np.zeros_like(theta0), np.zeros_like(theta0))
    ctx.set_eps_mode(0, seed=10)   # device Philox

    def orders(nb):
        rs = np.random.RandomState(15485863)  # VAEB.py:526 --seed default

        def order(n):
            out = []
            while len(out) < n:
                o = np.arange(nb)
                rs.shuffle(o)
                out.extend(o.tolist())
            return np.array(out[:n], np.int32)
        return order

    el, graph_modes = timed_run(ctx, orders(N // Bg), warmup, steps, dist, world, sync=args.sync,
                                warm_ms=args.device_warm_ms)
    elbo_sum, nsteps = ctx.epoch_elbo()
    comm = comm_record(ctx, dist, world)

    # per-kernel device time (HIP events on the context's stream), after the timed region
    prof = ctx.profile_steps(50 if not bf16 else 5)
    fl = phase_flops(D, H, Z, B, gaussian=gauss)
    if fv:   # the (mu, sigma) updates stream 32 B per parameter (FVS: + the gradient read and
        fl["fv_update"] = 32 * ctx.P   # the next step's sample written, Philox mode)
        fl["fvs_update"] = 40 * ctx.P
        fl["fvs_sample"] = 12 * ctx.P
    dom = max((k for k in prof if k[0] in fl), key=lambda k: k[1])
    traffic = committed_traffic(dom[0], PMC_FILES.get(args.config, ""))
    if dom[0] in ("fv_update", "fvs_update", "fvs_sample"):   # HBM-bound streams (config 4)
        achieved = fl[dom[0]] / (dom[1] * 1e-3) / 1e9
        peak, bound, unit = PEAK_HBM_GBS, "hbm", "GB/s"
    else:
        achieved = fl[dom[0]] / (dom[1] * 1e-3) / 1e12
        peak, bound, unit = (PEAK_BF16_TFLOPS if bf16 else PEAK_F32_TFLOPS), "mfma", "TFLOP/s"
    sflops = (fl["p1_enc_latent"] + fl["p4_decout_z"]) if C.get("estimator") == "FV" else \
        step_flops(D, H, Z, B, gaussian=gauss)

    res = {
        "metric": C["metric"],
        "value": Bg * steps / el,
        "unit": "images/s",
        "n_gpus": n_gpus,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": el / steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": C["dtype"],
        "data": (f"synthetic {'Bernoulli(0.5)' if bf16 else ('Frey-shaped Beta(2,2)' if gauss else 'MNIST-shaped binary')}"
                 f" pixels (N={N}, D={D}), "
                 f"resident in HBM; random init RandomState(10)"),
        "config": {"workload": C["workload"], "global_batch": Bg, "batch_per_gpu": B, "seq_len": None,
                   "parallelism": f"dp{world}"},
        "elbo": elbo_sum / max(nsteps, 1),
        "mode": "sync update(index) per step" if args.sync else "update_many (one call, graph replay)",
        "device_warm_ms": args.device_warm_ms,   # untimed busy kernel before the W warmup steps
        "graph": graph_modes,              # per rank: how the timed steps ran (vaeb_graph_status)
        "comm": comm,                      # per rank: RCCL version, overlap, algorithm / protocol
        "step_tflops": sflops / (el / steps) / 1e12,
        "kernels_ms": {k: round(v, 5) for k, v in prof},
        "roofline": {"bound": bound, "kernel": dom[0], "achieved": achieved, "peak": peak,
                     "unit": unit, "frac": achieved / peak, "traffic": traffic,
                     # traffic is not measured in this run: it is the committed rocprofv3 PMC pass
                     # (FETCH_SIZE x 2 + WRITE_SIZE per launch, MI355X_MICROARCH.md) of this build
                     "traffic_source": (os.path.relpath(PMC_FILES[args.config], ROOT)
                                        if traffic is not None else None),
                     ("bytes_per_launch" if bound == "hbm" else "flops_per_launch"): fl[dom[0]],
                     "avg_launch_ms": dom[1]},
    }
    ctx.close()
    if world > 1 and args.scaling == "weak" and not args.no_strong:
        # the same run with one Bn-row global minibatch split over the ranks
        Bs, off_s, Bgs = row_split(Bn, world, rank, "strong")
        ctx2 = make_context(C, D, H, Z, Bs, Bgs, off_s, local, args, gauss, bf16, dist, rank, world)
        ctx2.set_data(x)
        ctx2.set_params(theta0)
        ctx2.set_eps_mode(0, seed=10)
        el2, _ = timed_run(ctx2, orders(N // Bgs), warmup, steps, dist, world, warm_ms=args.device_warm_ms)
        ctx2.close()
        res["strong"] = {"value": Bgs * steps / el2, "ms_per_step": el2 / steps * 1e3, "global_batch": Bgs,
                         "rows_per_gpu": [row_split(Bn, world, r, "strong")[0] for r in range(world)]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if bf16:
            res["cpu_baseline"] = cpu_baseline(D, H, Z, B, x[:4 * B], budget_s=args.cpu_budget * 2, max_steps=8,
                                               single_kw={"max_steps": 1, "warm": 0})
        elif fv:
            res["cpu_baseline"] = cpu_baseline_fv(D, H, Z, B, x, budget_s=args.cpu_budget,
                                                  sample=C.get("estimator") == "FVS")
        else:
            res["cpu_baseline"] = cpu_baseline(D, H, Z, B, x, budget_s=args.cpu_budget, continuous=gauss)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
