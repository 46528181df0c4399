"""bench.py's data-parallel control flow on CPU (gloo, world size 2) with the HIP library
replaced by a recording stand-in: each rank builds its context with the weak-scaling row
split (rank r: rows [b*200 + 100 r, +100) of global minibatch b), checks the communicator
size, times its steps between barriers, and the strong-scaling leg re-splits one 100-row
minibatch 50 / 50; rank 0 prints one JSON line with n_gpus = 2."""
import io
import json
import os
import time
from contextlib import redirect_stdout

import pytest
import torch.multiprocessing as mp


class FakeCtx:
    made = []

    def __init__(self, D, H, Z, B, B_global=None, row_offset=0, device=0, **kw):
        self.cfg = dict(D=D, H=H, Z=Z, B=B, B_global=B_global, row_offset=row_offset, device=device)
        self.world, self.n, self.P = 1, 0, 1000
        FakeCtx.made.append(self.cfg)

    @staticmethod
    def comm_unique_id():
        return b"u" * 128

    def comm_init(self, uid, rank, world):
        assert len(uid) == 128
        self.world = world

    def comm_count(self):
        return self.world

    def set_data(self, x):
        self.rows = x.shape[0]

    def set_params(self, p):
        pass

    def set_fv_state(self, *a):
        pass

    def set_eps_mode(self, mode, seed=10):
        pass

    def update_many(self, order):
        assert order.max() < self.rows // self.cfg["B_global"]
        self.n += len(order)
        time.sleep(2e-5 * len(order))

    def synchronize(self):
        pass

    def epoch_elbo(self):
        n, self.n = self.n, 0
        return -100.0 * n, n

    def profile_steps(self, n):
        return [("p1_enc_latent", 0.012), ("p4_decout_z", 0.010)]

    def busy(self, us):
        assert us > 0

    def update(self, index):
        self.n += 1
        return -100.0

    def graph_status(self):
        if os.environ.get("FAKE_GRAPH_FAIL_RANK") == os.environ.get("RANK"):
            return "eager_fallback", "hipStreamEndCapture: operation not permitted when stream is capturing"
        return "replay", ""

    def comm_info(self):
        return {"rccl_version": 22700, "dp_overlap": False, "world": self.world}

    def close(self):
        pass


def _rank(rank, world, port, q, fail_rank=None):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    if fail_rank is not None:
        os.environ["FAKE_GRAPH_FAIL_RANK"] = str(fail_rank)
    import bench
    from vaeb_amd import _lib
    _lib.Context = FakeCtx
    buf = io.StringIO()
    try:
        with redirect_stdout(buf):
            bench.main(["--gpus", str(world), "--steps", "40", "--warmup", "4", "--no-cpu-baseline"])
    except SystemExit as e:
        q.put((rank, "exit", str(e.code)))
        raise
    q.put((rank, FakeCtx.made, buf.getvalue()))


def test_bench_two_ranks_weak_and_strong():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29900 + os.getpid() % 500
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(2):
        r, made, out = q.get(timeout=120)
        res[r] = (made, out)
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps)
    # weak: 100 rows per rank of a 200-row global minibatch; strong: 50 + 50 of 100
    assert res[0][0][0]["B"] == 100 and res[0][0][0]["B_global"] == 200 and res[0][0][0]["row_offset"] == 0
    assert res[1][0][0]["row_offset"] == 100 and res[1][0][0]["device"] == 1
    assert res[1][0][1]["B"] == 50 and res[1][0][1]["B_global"] == 100 and res[1][0][1]["row_offset"] == 50
    line = json.loads(res[0][1].strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["config"]["global_batch"] == 200
    assert line["graph"] == ["replay", "replay"]
    assert [c["dp_overlap"] for c in line["comm"]] == [False, False] and line["comm"][1]["algo"] == "auto"
    assert line["strong"]["rows_per_gpu"] == [50, 50] and line["strong"]["global_batch"] == 100
    assert line["value"] == pytest.approx(200 * 40 / (line["ms_per_step"] * 40 / 1e3), rel=1e-6)
    assert res[1][1].strip() == ""   # only rank 0 prints


def test_bench_fails_on_every_rank_when_one_rank_falls_back_to_eager():
    """at world > 1 a graph capture that fell back to eager launches must never
    be silent.  Rank 1's context reports the fallback after the warmup; bench gathers every
    rank's graph mode and all ranks exit non-zero (none is left waiting in a collective)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29900 + (os.getpid() + 250) % 500
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q, 1)) for r in range(2)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(2):
        r, kind, msg = q.get(timeout=120)
        got[r] = (kind, msg)
    for p in ps:
        p.join(60)
    assert all(p.exitcode not in (0, None) for p in ps), [p.exitcode for p in ps]
    assert all(k == "exit" and "rank(s) [1]" in m for k, m in got.values()), got
