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


def _shard_rank_main(rank, world, port, q):
    """Two steps of the sharded optimizer (vaeb_hip.hip dp_reduce_update) in torch.distributed
    (gloo): each rank's data gradient is summed and sliced to its shard (the reduce-scatter)
    and to the replicated remainders (the all-reduce); the rank applies the prior + Adagrad to
    its shard and the remainders only, keeping Adagrad state for those alone; the theta'
    shards are all-gathered.  Checked against the replicated update (every rank, the whole
    arena) on the oracle's decomposition: theta bit for bit on every rank, and the gathered
    Adagrad state equal to the replicated one."""
    from vaeb_amd.dp import arena_runs, shard_plan
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = O.Config(D=300, H=200, Z=20)
    shapes = [s for _, s in O.param_shapes(cfg)]
    offs = np.cumsum([0] + [int(np.prod(s)) for s in shapes])
    P = int(offs[-1])
    runs = arena_runs(offs, P)
    own, tails, foreign = shard_plan(runs, world, rank)
    assert own and tails and foreign
    mine = own + tails
    rng = np.random.default_rng(0)
    theta = np.concatenate([(rng.standard_normal(int(np.prod(s))) * 0.05) for s in shapes]).astype(np.float32)
    acc_rep = np.zeros(P, np.float32)
    theta_rep = theta.copy()
    acc_sh = np.zeros(P, np.float32)     # valid on this rank's own shard and the remainders only
    theta_sh = theta.copy()
    for step in range(2):
        xg = (np.random.default_rng(10 + step).random((24, cfg.D)) < 0.3).astype(np.float64)
        eps = np.random.default_rng(20 + step).standard_normal((1, 24, cfg.Z))
        rows = slice(12 * rank, 12 * rank + 12)
        out = O.forward_backward(O.unflatten(theta_sh.astype(np.float64), cfg), xg[rows], eps[:, rows], cfg)
        g = torch.tensor(np.concatenate([d.ravel() for d in out["data_grads"]]).astype(np.float32))
        dist.all_reduce(g)               # reduce-scatter + all-reduce, in one: each rank slices its part
        g = g.numpy()

        def rule(th, ac, gr):            # the float32 rule of kernels_aux.hpp opt_rule (prior 1)
            gg = (gr - th).astype(np.float32)
            ac = (ac + gg * gg).astype(np.float32)
            return (th + np.float32(cfg.lr) * gg / (np.sqrt(ac) + np.float32(1e-6))).astype(np.float32), ac

        theta_rep, acc_rep = rule(theta_rep, acc_rep, g)
        new = np.zeros(P, np.float32)
        for lo, n in mine:
            new[lo:lo + n], acc_sh[lo:lo + n] = rule(theta_sh[lo:lo + n], acc_sh[lo:lo + n], g[lo:lo + n])
        # the all-gather of the shards (the remainders are already everywhere)
        for lo, n in runs:
            S = (n // world) & ~63
            parts = [torch.zeros(S) for _ in range(world)]
            dist.all_gather(parts, torch.tensor(new[lo + rank * S:lo + (rank + 1) * S]))
            new[lo:lo + world * S] = torch.cat(parts).numpy()
        for lo, n in tails:
            assert np.array_equal(new[lo:lo + n], theta_rep[lo:lo + n])
        theta_sh = new
    # gather the Adagrad shards as vaeb_get_adagrad_state does (dp_gather_acc)
    for lo, n in runs:
        S = (n // world) & ~63
        parts = [torch.zeros(S) for _ in range(world)]
        dist.all_gather(parts, torch.tensor(acc_sh[lo + rank * S:lo + (rank + 1) * S]))
        acc_sh[lo:lo + world * S] = torch.cat(parts).numpy()
    q.put((rank, bool(np.array_equal(theta_sh, theta_rep)), bool(np.array_equal(acc_sh, acc_rep)),
           sum(n for _, n in own), P))
    dist.destroy_process_group()


def test_two_rank_sharded_optimizer_equals_replicated():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29300 + os.getpid() % 200
    procs = [ctx.Process(target=_shard_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, theta_ok, acc_ok, n_own, P in res:
        assert theta_ok and acc_ok, rank
        assert 0.45 * P <= n_own <= 0.5 * P     # each rank updates about half the arena itself


def test_shard_plan_covers_the_arena_once():
    """dp_opt_range / dp_foreign_range (mirrored by vaeb_amd.dp.shard_plan): for every world
    size, each rank's own shards + the replicated remainders + the foreign shards tile every
    run exactly once, the shards are 64-element aligned, and each element has one owner."""
    from vaeb_amd.dp import arena_runs, shard_plan
    for D, H, Z, gauss in ((784, 500, 20, False), (560, 200, 2, True), (4096, 2048, 128, False), (37, 19, 3, False)):
        cfg = O.Config(D=D, H=H, Z=Z, continuous=gauss)
        offs = np.cumsum([0] + [int(np.prod(s)) for _, s in O.param_shapes(cfg)])
        P = int(offs[-1])
        runs = arena_runs(offs, P, gauss)
        for world in (1, 2, 3, 8):
            owner = np.zeros(P, np.int32)
            for rank in range(world):
                own, tails, foreign = shard_plan(runs, world, rank)
                cover = np.zeros(P, np.int32)
                for lo, n in own + tails + foreign:
                    cover[lo:lo + n] += 1
                assert np.all(cover == 1), (D, world, rank)
                for lo, n in own:
                    assert lo % 64 == 0 or lo in [r[0] for r in runs] or (lo - [r[0] for r in runs if r[0] <= lo][-1]) % 64 == 0
                    owner[lo:lo + n] += 1
                if rank == 0:
                    tail_n = sum(n for _, n in tails)
                    assert tail_n <= 3 * 64 * world
            shard_n = owner.sum()
            assert np.all(owner <= 1) and shard_n >= P - 3 * 64 * world
