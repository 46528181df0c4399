"""The CLI's data-parallel path (DP and dtype at the drop-in surface), on CPU:
two gloo ranks run `cli.main([... '--world_size', '2'])` with the HIP library replaced by
a recording stand-in whose communicator is the gloo group itself.  Checked: the row split
of every minibatch (strong: the reference's 100-row minibatch as 50 + 50; weak: 100 per
rank), one RCCL id shared by both ranks, a single trace writer and printer (rank 0), the
same parameters on both ranks after training, and -- strong scaling -- the same
parameters and trace as the one-process run, since the ranks' rows tile each global
minibatch exactly (VAEB.py:340-344: the objective is a sum over rows)."""
import io
import os
from contextlib import redirect_stdout

import numpy as np
import pytest
import torch.multiprocessing as mp


class RecordingCtx:
    """Stand-in for vaeb_amd._lib.Context: a linear 'step' whose gradient is the sum of
    the rows this rank was given, all-reduced over the communicator (gloo here), then the
    same update on every rank -- the library's DP contract, without a GPU."""
    made = []

    def __init__(self, D, H, Z, B, L=1, decoder=0, estimator=0, objective=0, lr=0.01, adagrad_eps=1e-6, device=0,
                 B_global=None, row_offset=0, max_eval_rows=10000, use_graph=True, keep_grads=False, dtype=0):
        self.cfg = dict(D=D, H=H, Z=Z, B=B, B_global=B_global or B, row_offset=row_offset, device=device,
                        dtype=dtype)
        self.world, self.uid, self.steps, self.orders = 1, None, 0, []
        self.acc = [0.0, 0]
        RecordingCtx.made.append(self)

    @staticmethod
    def comm_unique_id():
        return os.urandom(128)

    def comm_init(self, uid, rank, world):
        assert len(uid) == 128
        self.uid, self.world = uid, world

    def comm_count(self):
        return self.world

    def _sum(self, v):
        if self.world == 1 or self.uid is None:
            return v
        import torch
        import torch.distributed as dist
        t = torch.tensor(v, dtype=torch.float64)
        dist.all_reduce(t)
        return t.numpy()

    def set_params(self, flat):
        self.theta = np.asarray(flat, np.float64).copy()
        self.P = self.theta.size

    def get_params(self):
        return self.theta.astype(np.float32)

    def set_data(self, x):
        self.x = np.asarray(x, np.float64)

    def set_eps_mode(self, mode, seed=10):
        pass

    def set_valid_data(self, x):
        self.xv = np.asarray(x, np.float64)

    def validate_resident(self):
        n = self.xv.shape[0]
        lo, hi = n * self.rank_share[0] // self.world, n * (self.rank_share[0] + 1) // self.world
        return float(self._sum(np.array([-self.xv[lo:hi].sum()]))[0])

    @property
    def rank_share(self):
        return (self.cfg["row_offset"] * self.world // self.cfg["B_global"],)

    def update_many(self, order):
        c = self.cfg
        for b in np.asarray(order).tolist():
            r0 = b * c["B_global"] + c["row_offset"]
            rows = self.x[r0:r0 + c["B"]]
            g = self._sum(np.concatenate([rows.sum(0), [rows.sum()]]))
            k = np.arange(self.P) % (g.size - 1)
            self.theta = self.theta - 1e-4 * g[k] + 1e-6 * np.sin(self.theta)
            self.acc[0] += -g[-1] / c["B_global"]
            self.acc[1] += 1
        self.orders.append(list(order))

    def epoch_elbo(self):
        out, self.acc = tuple(self.acc), [0.0, 0]
        return out

    def checkpoint_save(self, path):
        """vaeb_checkpoint_save under the sharded optimizer is a collective (the Adagrad shards
        are all-gathered before the write): modelled with a gloo all-gather every rank must
        join; path None = join without writing."""
        if self.world > 1 and self.uid is not None:
            import torch
            import torch.distributed as dist
            parts = [torch.zeros(4, dtype=torch.float64) for _ in range(self.world)]
            dist.all_gather(parts, torch.tensor(self.theta[:4]))
        if path is not None:
            with open(path, "w") as f:
                f.write("state")

    def close(self):
        pass


ARGV = ['--n_epochs', '2', '--synthetic', '--continuous', '--n_latent', '2', '--bogus', 'x']


def _run(argv):
    from vaeb_amd import _lib, cli
    real, _lib.Context = _lib.Context, RecordingCtx
    buf = io.StringIO()
    try:
        with redirect_stdout(buf):
            cli.main(argv)
    finally:
        _lib.Context = real
    m = RecordingCtx.made[-1]
    return m.cfg, m.uid, m.get_params(), [m.orders], buf.getvalue()


def _rank(rank, world, port, argv, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        q.put((rank,) + _run(argv))
    except BaseException as e:  # report, do not hang the parent
        q.put((rank, "error", repr(e), None, None, None))
        raise


def _two_ranks(argv):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29400 + os.getpid() % 400
    ps = [ctx.Process(target=_rank, args=(r, 2, port, argv, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(2):
        r, *rest = q.get(timeout=180)
        res[r] = rest
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps), res
    return res


@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_cli_world_size_two(tmp_path, monkeypatch, scaling):
    monkeypatch.chdir(tmp_path)
    trace = str(tmp_path / "t.csv")
    argv = ARGV + ['--trace_file', trace, '--world_size', '2', '--dp_scaling', scaling,
                   '--save_file', str(tmp_path / 'm.mdl'), '--state_file', str(tmp_path / 'm.state')]
    res = _two_ranks(argv)
    (c0, u0, th0, o0, out0), (c1, u1, th1, o1, out1) = res[0], res[1]
    if scaling == "strong":   # the reference's 100-row minibatch split 50 / 50
        assert (c0["B"], c0["B_global"], c0["row_offset"]) == (50, 100, 0)
        assert (c1["B"], c1["B_global"], c1["row_offset"]) == (50, 100, 50)
    else:                     # 100 rows per rank of a 200-row global minibatch
        assert (c0["B"], c0["B_global"], c0["row_offset"]) == (100, 200, 0)
        assert (c1["B"], c1["B_global"], c1["row_offset"]) == (100, 200, 100)
    assert c1["device"] == 1 and c0["device"] == 0
    assert u0 is not None and u0 == u1            # one RCCL id, drawn by rank 0
    assert o0 == o1                                # the same batch order on both ranks
    assert np.array_equal(th0, th1)                # replicas stay identical
    # rank 0 alone prints (the unused-argument report included) and writes the trace
    assert out0.count("Have unused args: ['--bogus', 'x']") == 1 and "Epoch 1 :" in out0
    assert out1 == ""
    rows = open(trace).read().splitlines()
    assert rows[0] == 'num_samples,L,Lvalid' and len(rows) == 5 and rows[1] == rows[2]
    assert os.path.exists(tmp_path / 'm.mdl')    # written once, by rank 0
    # the native checkpoint: a collective every rank joined, written by rank 0
    assert open(tmp_path / 'm.state').read() == "state"
    # the .mdl header holds the reference-level batch size (the global minibatch), not this
    # rank's share: strong 100, weak 200 rows per step
    from vaeb_amd.pickle_static import read_mdl
    hdr, _ = read_mdl(str(tmp_path / 'm.mdl'))
    assert int(hdr["batch_size"]) == (100 if scaling == "strong" else 200)
    if scaling == "strong":
        # the same steps as one process on the whole minibatch
        monkeypatch.delenv("WORLD_SIZE", raising=False)
        c, u, th, o, out = _run(ARGV + ['--trace_file', str(tmp_path / 't1.csv')])
        assert u is None and c["B"] == 100
        np.testing.assert_allclose(th, th0, rtol=1e-6, atol=1e-6)
        one = [[float(v) for v in r.split(',')] for r in open(tmp_path / 't1.csv').read().splitlines()[1:]]
        two = [[float(v) for v in r.split(',')] for r in rows[1:]]
        np.testing.assert_allclose(one, two, rtol=1e-12)


def test_cli_world_size_one_takes_a_communicator(tmp_path, monkeypatch):
    """--world_size 1: the data-parallel step (all-reduce + optimizer launch) on one GPU;
    the default (0) keeps the fused single-GPU step without a communicator."""
    monkeypatch.chdir(tmp_path)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    c, u, _, _, out = _run(ARGV + ['--world_size', '1'])
    assert u is not None and (c["B"], c["B_global"], c["row_offset"]) == (100, 100, 0)
    c, u, _, _, _ = _run(ARGV)
    assert u is None


def test_cli_dtype_key(tmp_path, monkeypatch):
    from vaeb_amd import _lib
    from vaeb_amd.model import dtype_name
    monkeypatch.chdir(tmp_path)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    c, _, _, _, out = _run(ARGV + ['--dtype', 'bf16'])
    assert c["dtype"] == _lib.DTYPE_BF16 and "\tdtype: bf16" in out
    c, _, _, _, _ = _run(ARGV)
    assert c["dtype"] == _lib.DTYPE_F32
    assert dtype_name("float32") == "float32" and dtype_name("bfloat16") == "bf16"
    assert dtype_name("float16") == "fp16" and dtype_name("half") == "fp16"
    c, _, _, _, out = _run(ARGV + ['--dtype', 'float16'])
    assert c["dtype"] == _lib.DTYPE_F16
    with pytest.raises(ValueError):
        dtype_name("int8")


def test_cli_world_size_must_match_the_launcher(monkeypatch):
    from vaeb_amd import cli
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "0")
    with pytest.raises(ValueError, match="launcher started 4"):
        cli.dp_layout({'world_size': 2})
    assert cli.dp_layout({'world_size': 0})[:2] == (4, 0)
