"""Data-parallel decomposition of the SGVB step, checked with real torch.distributed
(gloo, world_size 2, CPU).  This is the host orchestration the HIP path implements with
one RCCL all-reduce per step (vaeb_hip.hip: P8 grads -> ncclAllReduce([grads | SGVB]) ->
adagrad_kernel): every rank computes the data gradient of its rows, the SUM is
all-reduced, the -theta prior is added once after the reduce, and every rank applies the
identical Adagrad update.  The result must equal the single-process step on the
concatenated global batch (VAEB.py:340-344: the objective is a sum over rows)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import vaeb_oracle as O
from vaeb_amd.dp import row_split


def _rank_main(rank, world, port, mode, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = O.Config(D=40, H=24, Z=5, L=2 if mode == "L2" else 1,
                   continuous=(mode == "gauss"), estimator="LA" if mode == "LA" else "LB")
    # weak scaling: 12 rows per rank; strong: a 25-row global batch split 13 / 12
    B, off, Bg = row_split(25 if mode == "strong" else 12, world, rank, "strong" if mode == "strong" else "weak")
    rng = np.random.default_rng(0)
    params = [(rng.standard_normal(s) * 0.2).astype(np.float64) for _, s in O.param_shapes(cfg)]
    xg = rng.random((Bg, cfg.D))
    if not cfg.continuous:
        xg = (xg < 0.4).astype(np.float64)
    epsg = rng.standard_normal((cfg.L, Bg, cfg.Z))
    rows = slice(off, off + B)
    out = O.forward_backward(params, xg[rows], epsg[:, rows], cfg)
    flat = torch.tensor(np.concatenate([g.ravel() for g in out["data_grads"]] + [[out["sgvb"]]]))
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    red = flat.numpy()
    grads = O.unflatten(red[:-1], cfg)
    grads = [g - p for g, p in zip(grads, params)]  # prior once, after the reduce
    acc = [np.zeros_like(p) for p in params]
    newp, _ = O.adagrad_update(params, acc, grads, cfg)
    if rank == 0:
        full = O.forward_backward(params, xg, epsg, cfg)
        ref_p, _ = O.adagrad_update(params, acc, full["grads"], cfg)
        q.put((float(red[-1]), float(full["sgvb"]),
               max(float(np.abs(a - b).max()) for a, b in zip(newp, ref_p))))
    # every rank must hold bit-identical parameters after the replicated update
    mine = torch.tensor(np.concatenate([p.ravel() for p in newp]))
    other = mine.clone()
    dist.broadcast(other, src=0)
    assert torch.equal(mine, other)
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["LB", "LA", "gauss", "L2", "strong"])
def test_two_rank_allreduce_equals_global_step(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (abs(hash(mode)) % 2000)
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    sg_red, sg_full, dtheta = q.get(timeout=5)
    assert abs(sg_red - sg_full) <= 1e-9 * abs(sg_full)
    assert dtheta <= 1e-12


def test_weak_scaling_row_map():
    """bench.py / vaeb_config: rank r of world W takes rows
    [b * B * W + r * B, b * B * W + (r + 1) * B) of global minibatch b."""
    B, W, b = 100, 8, 17
    cover = np.concatenate([np.arange(b * B * W + r * B, b * B * W + (r + 1) * B) for r in range(W)])
    assert np.array_equal(cover, np.arange(b * B * W, (b + 1) * B * W))


def test_strong_scaling_row_map():
    """bench.py --scaling strong: a 100-row global minibatch over 8 ranks is
    13,13,13,13,12,12,12,12 contiguous rows, covering it exactly once."""
    parts = [row_split(100, 8, r, "strong") for r in range(8)]
    assert [p[0] for p in parts] == [13, 13, 13, 13, 12, 12, 12, 12]
    assert all(p[2] == 100 for p in parts)
    cover = np.concatenate([np.arange(off, off + n) for n, off, _ in parts])
    assert np.array_equal(cover, np.arange(100))
    with pytest.raises(ValueError):
        row_split(4, 8, 0, "strong")
