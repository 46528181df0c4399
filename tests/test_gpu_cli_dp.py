"""The CLI's data-parallel and dtype keys on the GPU (the (b) CLI row): one rank
with a communicator (`--world_size 1`: the all-reduce step), on the bf16 engine
(`--dtype bf16`) at a reduced shape, against the oracle with bf16 rounding at the engine's
rounding points; and the fp32 DP step through the CLI against the default fused step.

Tolerances (the bf16 parity suite's, tests/test_gpu_bf16.py): ELBO 1e-4 relative per
epoch of the first epoch's steps, 5e-4 after a further epoch and for the validation bound
(bf16 rounding ties can flip as the trajectories move apart by fp32 accumulation order);
parameters norm-wise 1e-3."""
import numpy as np
import pytest

from oracle import vaeb_oracle as O

pytestmark = pytest.mark.gpu


def _rows(path):
    return [[float(v) for v in r.split(',')] for r in open(path).read().splitlines()[1:]]


def _clean_env(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)


def test_cli_world1_communicator_bf16_matches_rounded_oracle(tmp_path, monkeypatch):
    from vaeb_amd import cli
    from vaeb_amd.model import TheanoStreamEmulation
    _clean_env(monkeypatch)
    monkeypatch.chdir(tmp_path)
    x = O.synthetic_mnist(n=768, seed=4)
    monkeypatch.setattr(cli, "load_dataset", lambda continuous, synthetic=False, splits=2: (x[:512], x[512:]))
    trace = str(tmp_path / "t.csv")
    model, _ = cli.main(['--n_epochs', '2', '--world_size', '1', '--dtype', 'bf16', '--hidden_unit', '64',
                         '--n_latent', '16', '--batch_size', '128', '--rng', 'theano', '--trace_file', trace,
                         '--trace_dedup', '1'])
    assert model._ctx.comm_count() == 1 and model.dtype == "bf16"
    theta = model._ctx.get_params()
    model.close()

    cfg = O.Config(D=784, H=64, Z=16)
    p = [a.astype(np.float64) for a in O.init_params(cfg)]
    acc = [np.zeros_like(a) for a in p]
    stream = TheanoStreamEmulation(1, 10)
    np.random.seed(15485863)               # VAEB.py:526 (--seed default), then one shuffle per epoch
    order = np.arange(4)
    want = []
    for epoch in range(2):
        np.random.shuffle(order)
        lb = 0.0
        for b in order:
            eps = stream.draw(128, 16).astype(np.float64)
            v, p, acc, _ = O.step(p, acc, x[b * 128:(b + 1) * 128].astype(np.float64), eps, cfg, q=O.bf16_round)
            lb += v
        ev = stream.draw(256, 16).astype(np.float64)
        want.append([512 * (epoch + 1), lb / 4, O.validate(p, x[512:].astype(np.float64), ev, cfg, q=O.bf16_round) / 256])
    got = _rows(trace)
    assert [r[0] for r in got] == [w[0] for w in want]
    assert abs(got[0][1] - want[0][1]) <= 1e-4 * abs(want[0][1]), (got, want)
    for g, w in zip(got, want):
        assert abs(g[1] - w[1]) <= 5e-4 * abs(w[1]) and abs(g[2] - w[2]) <= 5e-4 * abs(w[2]), (got, want)
    ref = O.flatten(p)
    assert np.linalg.norm(theta - ref) <= 1e-3 * np.linalg.norm(ref)


def test_cli_world1_communicator_fp32_equals_fused_step(tmp_path, monkeypatch):
    """fp32 MNIST 784-500-20 through the CLI: `--world_size 1` (all-reduce + optimizer
    launch) against the default fused-optimizer step, same Philox noise: the same trace."""
    from vaeb_amd import cli
    _clean_env(monkeypatch)
    monkeypatch.chdir(tmp_path)
    x = O.synthetic_mnist(n=1500, seed=2)
    monkeypatch.setattr(cli, "load_dataset", lambda continuous, synthetic=False, splits=2: (x[:1200], x[1200:]))
    rows = []
    for extra in ([], ['--world_size', '1']):
        t = str(tmp_path / f"t{len(rows)}.csv")
        model, _ = cli.main(['--n_epochs', '2', '--n_latent', '20', '--trace_file', t, '--trace_dedup', '1'] + extra)
        # dp_overlap is None without a communicator (vaeb_comm_info)
        assert (model._ctx.comm_info()["dp_overlap"] is not None) == bool(extra)
        model.close()
        rows.append(_rows(t))
    np.testing.assert_allclose(rows[0], rows[1], rtol=1e-6)


@pytest.mark.parametrize("dtype", ["float32", "bf16"])
def test_cli_world1_sharded_optimizer_equals_replicated(tmp_path, monkeypatch, dtype):
    """the sharded DP optimizer (reduce-scatter -> own-shard Adagrad ->
    all-gather, VAEB_DP_SHARD=1) through cli.main at --world_size 1, against the replicated
    all-reduce + Adagrad (VAEB_DP_SHARD=0): the same trace, parameters and native checkpoint
    (--state_file: the Adagrad shards gathered before the write), bit for bit."""
    from vaeb_amd import cli
    _clean_env(monkeypatch)
    monkeypatch.chdir(tmp_path)
    x = O.synthetic_mnist(n=1500, seed=3)
    monkeypatch.setattr(cli, "load_dataset", lambda continuous, synthetic=False, splits=2: (x[:1200], x[1200:]))
    shape = ['--n_latent', '20'] if dtype == "float32" else ['--hidden_unit', '64', '--n_latent', '16',
                                                              '--batch_size', '120']
    out = {}
    for shard in ("1", "0"):
        monkeypatch.setenv("VAEB_DP_SHARD", shard)
        t = str(tmp_path / f"t{shard}.csv")
        st = str(tmp_path / f"s{shard}.ckpt")
        model, _ = cli.main(['--n_epochs', '2', '--world_size', '1', '--dtype', dtype, '--trace_file', t,
                             '--trace_dedup', '1', '--state_file', st] + shape)
        assert model._ctx.comm_count() == 1
        out[shard] = (_rows(t), model._ctx.get_params(), open(st, "rb").read())
        model.close()
    assert out["1"][0] == out["0"][0]
    assert np.array_equal(out["1"][1], out["0"][1])
    assert out["1"][2] == out["0"][2]
