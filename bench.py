#!/usr/bin/env python3
"""Benchmark: SGVB training images/sec + ELBO at MNIST 784-500-20, batch 100 per GPU.

A "step" is one VAEB.update (/root/reference/VAEB.py:408-415) on one minibatch of 100
synthetic MNIST-shaped rows: encoder -> reparameterised sample -> decoder -> ELBO + KL ->
gradient -> Adagrad, all on the GPU (libvaeb_hip.so); the training set is resident in
HBM before timing starts.  With N GPUs every rank processes its own 100 rows of a
100*N-row global minibatch and the gradients are all-reduced over RCCL ("weak" scaling).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
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

PEAK_F32_TFLOPS = 157.3   # MI355X f32 MFMA / vector peak (MI355X_MICROARCH.md)
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
    }


KERNEL_SYMBOLS = {"p1_enc": "PEnc", "p23_heads_dechid": "heads_dechid_kernel", "p4_decout": "PDecOut",
                  "p5_dhd_w2": "vaeb::tile_wgrad_kernel", "p67_dz_dh_w1": "vaeb::dz_dh_wgrad_kernel",
                  "p8_wgrad_w3w45": "vaeb::wgrad_kernel", "p1_enc_latent": "vaeb::enc_latent_kernel",
                  "p4_decout_z": "vaeb::decout_z_kernel"}
PMC_FILE = os.path.join(ROOT, "profiles", "r1", "pmc_per_launch.json")


def committed_traffic(kernel, path=PMC_FILE, symbols=KERNEL_SYMBOLS):
    """HBM bytes per launch of `kernel` from the rocprofv3 PMC passes committed under
    profiles/ (separate FETCH_SIZE / WRITE_SIZE passes folded by scripts/pmc_summary.py,
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM)."""
    try:
        data = json.load(open(path))
    except Exception:
        return None
    sym = symbols.get(kernel)
    for name, v in data.items():
        if sym and sym in name and "hbm_bytes_per_launch" in v:
            return v["hbm_bytes_per_launch"]
    return None


def cpu_baseline(D, H, Z, B, x, budget_s=10.0):
    """The oracle's float32 NumPy restatement of the same step, on the host cores."""
    from oracle import vaeb_oracle as O
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    threads = min(16, os.cpu_count() or 1)
    cfg = O.Config(D=D, H=H, Z=Z)
    params = O.init_params(cfg)
    acc = [np.zeros_like(p) for p in params]
    rng = np.random.default_rng(0)
    nb = x.shape[0] // B
    ctx = threadpool_limits(limits=threads) if threadpool_limits else None
    try:
        for i in range(3):  # warm-up
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
            if dt >= budget_s or n >= 20000:
                break
    finally:
        if ctx is not None:
            ctx.unregister() if hasattr(ctx, "unregister") else None
    return {"value": n * B / dt, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} float32 NumPy oracle steps (784-500-20, B={B}) in {dt:.1f} s, OpenBLAS {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {args.gpus}", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist  # host-side coordination only (gloo)
        dist.init_process_group("gloo")

    from oracle import vaeb_oracle as O  # synthetic data generator + initial theta (not the compute path)
    from vaeb_amd import _lib

    D, H, Z, B = 784, 500, 20, args.batch
    Bg = B * world
    N = 50000
    x = O.synthetic_mnist(n=N, D=D)
    cfg = O.Config(D=D, H=H, Z=Z)
    ctx = _lib.Context(D, H, Z, B, B_global=Bg, row_offset=rank * B, device=local,
                       use_graph=not args.no_graph, max_eval_rows=1000)
    if world > 1:
        uid = [_lib.Context.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(uid[0], rank, world)
    ctx.set_data(x)
    ctx.set_params(O.flatten(O.init_params(cfg)))
    ctx.set_eps_mode(_lib.EPS_PHILOX, seed=10)
    nb = N // Bg
    rs = np.random.RandomState(15485863)  # VAEB.py:526 --seed default

    def order(n):
        out = []
        while len(out) < n:
            o = np.arange(nb)
            rs.shuffle(o)
            out.extend(o.tolist())
        return np.array(out[:n], np.int32)

    ctx.update_many(order(args.warmup))
    ctx.synchronize()
    ctx.epoch_elbo()
    timed_order = order(args.steps)
    if dist:
        dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
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
    elbo_sum, nsteps = ctx.epoch_elbo()

    # per-kernel device time (HIP events on the context's stream), after the timed region
    prof = ctx.profile_steps(50)
    fl = phase_flops(D, H, Z, B)
    dom = max((k for k in prof if k[0] in fl), key=lambda k: k[1])
    achieved = fl[dom[0]] / (dom[1] * 1e-3) / 1e12
    traffic = committed_traffic(dom[0])

    res = {
        "metric": "SGVB training images/sec + ELBO at MNIST 784-500-20, batch 100",
        "value": world * B * args.steps / el,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic MNIST-shaped binary pixels (N={N}, D={D}), resident in HBM; random init RandomState(10)",
        "config": {"workload": "MNIST 784-500-20 Bernoulli decoder, LB estimator, L=1, Adagrad lr 0.01",
                   "global_batch": Bg, "batch_per_gpu": B, "seq_len": None, "parallelism": f"dp{world}"},
        "elbo": elbo_sum / max(nsteps, 1),
        "kernels_ms": {k: round(v, 5) for k, v in prof},
        "roofline": {"bound": "mfma", "kernel": dom[0], "achieved": achieved, "peak": PEAK_F32_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / PEAK_F32_TFLOPS, "traffic": traffic,
                     "flops_per_launch": fl[dom[0]], "avg_launch_ms": dom[1]},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(D, H, Z, B, x, budget_s=args.cpu_budget)
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
