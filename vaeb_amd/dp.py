"""Data parallelism on the host side: the row partition of a global minibatch,
the rank launcher, and the RCCL communicator set-up.

The SGVB objective is a sum over batch rows (VAEB.py:340-344), so a step shards by rows:
rank r takes a contiguous block of the global minibatch and the gradients are summed with
one all-reduce inside the library (RCCL over xGMI).  Weak scaling gives every rank B rows
(B_global = B * world); strong scaling splits a fixed global batch as evenly as possible,
earlier ranks taking the remainder (100 over 8 ranks = 13,13,13,13,12,12,12,12).

One process per GPU: ranks come from RANK / LOCAL_RANK / WORLD_SIZE, set by a launcher
(torch.distributed.run) or by `spawn_ranks` before any GPU call.  torch.distributed (gloo)
is host-side coordination only: it carries the 128-byte RCCL id from rank 0 to the others.
"""
from __future__ import annotations

import os
import subprocess
import sys
import time


def row_split(batch, world, rank, scaling="weak"):
    """Returns (rows of this rank, its row offset inside the global minibatch, B_global)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    if scaling == "weak":
        return batch, rank * batch, batch * world
    if scaling != "strong":
        raise ValueError(f"unknown scaling {scaling!r}")
    if batch < world:
        raise ValueError(f"strong scaling needs at least one row per rank ({batch} rows, {world} ranks)")
    base, extra = divmod(batch, world)
    rows = [base + (1 if r < extra else 0) for r in range(world)]
    return rows[rank], sum(rows[:rank]), batch


def env_ranks():
    """(world, rank, local_rank) from the launcher's environment (1, 0, 0 without one)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


RANK_HUNG = 124   # spawn_ranks: a rank still running after its peers finished (timeout(1)'s code)


def spawn_ranks(n, cmd, poll_s=0.2, env_extra=None, straggler_s=None):
    """Start n rank processes of `cmd` (an argv list; one per GPU, RANK = LOCAL_RANK = r,
    WORLD_SIZE = n, rendezvous on 127.0.0.1) and wait.  The parent makes no GPU call.  If
    one rank fails the others are stopped (they would wait in a collective forever);
    returns the first non-zero exit code, else 0.  Once any rank has exited 0 the others get
    `straggler_s` seconds (VAEB_RANK_DEADLINE_S, default 600) to follow: a rank left alone in a
    collective would otherwise hold the launcher forever.  Past it they are killed, the
    still-running ranks are named on stderr, and the code is RANK_HUNG.  (cli.train_model ends
    with a barrier of all ranks after rank 0's lead-only work -- the .mdl, the trace -- so healthy
    ranks exit together and the deadline never runs against that tail.)"""
    if straggler_s is None:
        straggler_s = float(os.environ.get("VAEB_RANK_DEADLINE_S", "600"))
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **(env_extra or {}))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen(list(cmd), env=env))

    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()

    first_done = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            stop_all()
            return bad[0]
        if all(c == 0 for c in codes):
            return 0
        if first_done is None and any(c == 0 for c in codes):
            first_done = time.monotonic()
        if first_done is not None and time.monotonic() - first_done > straggler_s:
            hung = [r for r, c in enumerate(codes) if c is None]
            print(f"spawn_ranks: rank(s) {hung} still running {straggler_s:g} s after a peer finished; "
                  f"stopping them", file=sys.stderr, flush=True)
            stop_all()
            return RANK_HUNG
        time.sleep(poll_s)


def module_cmd(argv):
    """`python -m vaeb_amd <argv>` with this interpreter (the CLI's rank processes)."""
    return [sys.executable, "-m", "vaeb_amd"] + list(argv)


def init_host_group(world):
    """The gloo process group the ranks coordinate on (None at world 1)."""
    if world <= 1:
        return None
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    return dist


def comm_uid(dist, rank, unique_id):
    """The RCCL id every rank passes to vaeb_comm_init: drawn by rank 0 (unique_id()), carried
    to the others over the gloo group (dist None: world 1, no broadcast)."""
    uid = [unique_id() if rank == 0 else None]
    if dist is not None:
        dist.broadcast_object_list(uid, src=0)
    return uid[0]


def comm_setup(ctx, dist, rank, world):
    """The library's RCCL communicator for `ctx` (vaeb_comm_init): rank 0 draws the id, the
    gloo group carries it.  At world 1 (dist None) a one-rank communicator: the data-parallel
    step (all-reduce + Adagrad launch) on one GPU.  Checks ncclCommCount == world."""
    if dist is None and world != 1:
        raise ValueError("world > 1 needs the host process group")
    ctx.comm_init(comm_uid(dist, rank, type(ctx).comm_unique_id), rank, world)
    n = ctx.comm_count()
    if n != world:
        raise RuntimeError(f"rank {rank}: the RCCL communicator holds {n} ranks, expected {world}")
    return n


def arena_runs(offsets, P, gaussian=False):
    """The three runs the DP optimizer partitions the parameter arena into (vaeb_hip.hip
    dp_bucket_all_runs): B0 = [0, W2), A = [W2, b3) (W2 | W6), B1 = [b3, P); `offsets` are
    the arena offsets in reference order (W3 W4 W5 W1 W2 [W6] b3 ...)."""
    bo = 6 if gaussian else 5
    return [(0, offsets[4]), (offsets[4], offsets[bo] - offsets[4]), (offsets[bo], P - offsets[bo])]


def shard_len(n, world, sharded=True):
    """Elements per rank of a run of n (vaeb_hip.hip dp_shard_len): 64-aligned floor(n / world)."""
    return (n // world) & ~63 if sharded else 0


def shard_plan(runs, world, rank, sharded=True):
    """Host mirror of the sharded optimizer's index plan (vaeb_hip.hip dp_reduce_update,
    dp_opt_range, dp_foreign_range), for tests and the cost model.  Per run (lo, n):
    reduce-scatter of world * S elements (this rank's shard [lo + rank S, +S)), all-reduce of
    the remainder [lo + world S, lo + n); the optimizer updates the shard and the remainder;
    the all-gather brings the other ranks' shards.  Returns (own, tails, foreign) as lists of
    (lo, n) index runs."""
    own, tails, foreign = [], [], []
    for lo, n in runs:
        S = shard_len(n, world, sharded)
        if S:
            own.append((lo + rank * S, S))
            if rank > 0:
                foreign.append((lo, rank * S))
            if rank < world - 1:
                foreign.append((lo + (rank + 1) * S, (world - rank - 1) * S))
        if n - world * S:
            tails.append((lo + world * S, n - world * S))
    return own, tails, foreign
