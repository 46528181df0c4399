"""GPU tests of the drop-in surfaces above the kernels: the VAEB class (VAEB.py:132-242
contract), the CLI main() on synthetic data, and the data-parallel code path (RCCL
communicator + all-reduce + replicated Adagrad) at world size 1 on the test box."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import vaeb_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_vaeb_class_update_validate_save_load(tmp_path):
    from vaeb_amd.model import VAEB
    x = O.synthetic_mnist(n=1200)
    xv = O.synthetic_mnist(n=300, seed=7)
    m = VAEB(x, False, 500, 20, 100, 1, 0.01, False, False)
    assert m.N == 1200 and m.batch_size == 100 and m.n_latent == 20
    assert [p.name for p in m.params] == ["W3", "W4", "W5", "W1", "W2", "b3", "b4", "b5", "b1", "b2"]
    p0 = [p.get_value() for p in m.params]
    assert np.array_equal(p0[0], O.init_params(O.Config(D=784, H=500, Z=20))[0])
    e = [m.update(i) for i in range(12)]
    assert all(np.isfinite(e)) and e[-1] > e[0]  # the bound improves over 12 steps
    v = m.validate(xv)
    assert np.isfinite(v) and v < 0
    f = tmp_path / "m.mdl"
    m.save(str(f))
    m2, _ = VAEB.load(str(f), data=(x, xv))
    assert all(np.array_equal(a.get_value(), b.get_value()) for a, b in zip(m.params, m2.params))
    s = m.update_epoch(np.arange(12))
    assert np.isfinite(s)
    y = m.reconstruct(xv[:10])
    assert y.shape == (10, 784) and np.all((y > 0) & (y < 1))


def test_vaeb_class_theano_rng_mode_is_reproducible():
    from vaeb_amd.model import VAEB
    x = O.synthetic_frey(n=600)
    r = []
    for _ in range(2):
        m = VAEB(x, True, 200, 2, 100, 1, 0.01, False, False, rng="theano")
        r.append([m.update(i % 6) for i in range(6)] + [m.validate(x[:100])])
        m.close()
    assert r[0] == r[1]


@pytest.mark.parametrize("continuous,use_graph,overlap,shard", [
    (False, True, "1", "0"), (True, True, "1", "0"), (False, False, "1", "0"), (False, True, "0", "0"),
    (True, True, "0", "0"),
    # the sharded optimizer (reduce-scatter -> own shard of Adagrad -> all-gather), forced at world 1
    (False, True, "0", "1"), (True, True, "1", "1"), (False, False, "1", "1")])
def test_dp_path_world1_matches_fused_path(continuous, use_graph, overlap, shard, monkeypatch):
    """The data-parallel path (gradients stored; with VAEB_DP_OVERLAP=1 -- the bf16 engine's
    default -- bucket A = W2 [| W6] all-reduced and updated on the second stream while the
    backward continues, bucket B + SGVB after it; with 0 -- the fp32 default -- one
    all-reduce and one optimizer launch) at world size 1 against the fused-optimizer path:
    Bernoulli / Gaussian decoder, graph-replayed and eager."""
    from vaeb_amd import _lib
    monkeypatch.setenv("VAEB_DP_OVERLAP", overlap)
    monkeypatch.setenv("VAEB_DP_SHARD", shard)
    cfg = O.Config(D=560, H=200, Z=2, continuous=True) if continuous else O.Config(D=784, H=500, Z=20)
    x = O.synthetic_frey(n=2000) if continuous else O.synthetic_mnist(n=2000)
    order = np.random.default_rng(1).permutation(20).astype(np.int32)
    outs = []
    for use_comm in (False, True):
        ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, 100, max_eval_rows=500, use_graph=use_graph,
                           decoder=_lib.DEC_GAUSSIAN if continuous else _lib.DEC_BERNOULLI)
        if use_comm:
            ctx.comm_init(_lib.Context.comm_unique_id(), 0, 1)
            assert ctx.comm_info()["dp_overlap"] == (overlap == "1")
        ctx.set_data(x)
        ctx.set_params(O.flatten(O.init_params(cfg)))
        ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
        ctx.set_step(0)
        ctx.update_many(order)
        assert ctx.graph_status()[0] == ("replay" if use_graph else "off")
        s, n = ctx.epoch_elbo()
        outs.append((s, ctx.get_params(), ctx.get_adagrad_state()))
        ctx.close()
    assert abs(outs[0][0] - outs[1][0]) <= 1e-6 * abs(outs[0][0])
    assert np.abs(outs[0][1] - outs[1][1]).max() <= 1e-6
    assert np.abs(outs[0][2] - outs[1][2]).max() <= 1e-3 * np.abs(outs[0][2]).max()


def test_cli_main_synthetic(tmp_path):
    trace = tmp_path / "trace.csv"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "VAEB.py"), "--n_latent", "20", "--n_epochs", "2",
                        "--synthetic", "--trace_file", str(trace)], capture_output=True, text=True, cwd=tmp_path,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Epoch 1 : [Lower bound:" in r.stdout
    rows = trace.read_text().splitlines()
    assert rows[0] == "num_samples,L,Lvalid" and len(rows) == 5
    lb = [float(x.split(",")[1]) for x in rows[1:]]
    assert lb[2] > lb[0]  # epoch 2 better than epoch 1


def test_vaeb_class_fv_weight_sampling_extension():
    """VAEB(..., fullVariational=True, fv_sample=True): theta~ = mu + |sigma| zeta each step
    (VAEB.py:127-129); reproducible in the host-noise ('theano') mode, the loaded theta
    untouched, the variational parameters moving."""
    from vaeb_amd.model import VAEB
    x = O.synthetic_frey(n=600)
    theta = O.init_params(O.Config(D=560, H=200, Z=2, continuous=True))
    runs = []
    for _ in range(2):
        m = VAEB(x, True, 200, 2, 100, 1, 0.01, False, True, params=theta, rng="theano", fv_sample=True)
        e = [m.update(i % 6) for i in range(6)]
        assert all(np.isfinite(e))
        fvp = m.full_variational_params
        runs.append((e, fvp[0].copy()))
        assert all(np.array_equal(p.get_value(), t) for p, t in zip(m.params, theta))
        assert not np.array_equal(fvp[0], theta[0])
        m.close()
    assert runs[0][0] == runs[1][0] and np.array_equal(runs[0][1], runs[1][1])


def test_vaeb_optimizer_plugin_binds_the_engine_rule():
    """inf=AdaGrad(eta) (degenerate-vae/infalg.py contract): eta becomes the engine's step
    size, and the accumulators construct() hands out are views of the engine's arena."""
    from vaeb_amd.infalg import AdaGrad
    from vaeb_amd.model import VAEB
    x = O.synthetic_mnist(n=400)
    a = VAEB(x, False, 500, 20, 100, 1, 0.01, False, False, inf=AdaGrad(0.03))
    b = VAEB(x, False, 500, 20, 100, 1, 0.03, False, False)
    assert a.update(0) == b.update(0)
    assert all(np.array_equal(p.get_value(), q.get_value()) for p, q in zip(a.params, b.params))
    acc = a.updates[0][0]
    assert np.array_equal(acc.get_value(), a.ADA[0])
    acc.set_value(np.zeros_like(a.ADA[0]))
    assert not a.ADA[0].any() and a.ADA[1].any()


@pytest.mark.parametrize("continuous,overlap", [(False, "0"), (True, "1"), (False, "1")])
def test_sharded_dp_optimizer_world1_is_bitwise_the_replicated_one(continuous, overlap, monkeypatch):
    """the sharded DP optimizer (vaeb_hip.hip dp_reduce_update: reduce-scatter of
    each arena run's 64-aligned shards + all-reduce of the remainders and the SGVB slot, this
    rank's shard of prior + Adagrad, all-gather of theta' shards) forced at world 1 equals the
    replicated DP path (all-reduce, Adagrad over the whole arena) bit for bit: ELBO, theta and
    the Adagrad state, graph-replayed and eager, with bucket A overlapped or not."""
    from vaeb_amd import _lib
    monkeypatch.setenv("VAEB_DP_OVERLAP", overlap)
    cfg = O.Config(D=560, H=200, Z=2, continuous=True) if continuous else O.Config(D=784, H=500, Z=20)
    x = O.synthetic_frey(n=2000) if continuous else O.synthetic_mnist(n=2000)
    order = np.random.default_rng(2).permutation(20).astype(np.int32)
    outs = {}
    for shard in ("0", "1"):
        for use_graph in (True, False):
            monkeypatch.setenv("VAEB_DP_SHARD", shard)
            ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, 100, max_eval_rows=500, use_graph=use_graph,
                               decoder=_lib.DEC_GAUSSIAN if continuous else _lib.DEC_BERNOULLI)
            ctx.comm_init(_lib.Context.comm_unique_id(), 0, 1)
            ctx.set_data(x)
            ctx.set_params(O.flatten(O.init_params(cfg)))
            ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
            ctx.update_many(order)
            v = ctx.update(3)
            s, n = ctx.epoch_elbo()
            outs[shard, use_graph] = (s, v, ctx.get_params(), ctx.get_adagrad_state())
            ctx.close()
    ref = outs["0", True]
    for key, o in outs.items():
        assert o[0] == ref[0] and o[1] == ref[1], key
        assert np.array_equal(o[2], ref[2]) and np.array_equal(o[3], ref[3]), key


@pytest.mark.parametrize("shard", ["0", "1"])
def test_dp_eager_update_matches_graph_update_many(shard, monkeypatch):
    """vaeb_update runs its step eagerly at any world size (and update_many's
    first step is eager too), so the eager data-parallel step is a product path: with a
    communicator (world 1; the sharded optimizer forced or not) one update(i) per batch
    equals update_many(order) over graph replay bit for bit -- ELBO, theta, Adagrad state."""
    from vaeb_amd import _lib
    monkeypatch.setenv("VAEB_DP_SHARD", shard)
    cfg = O.Config(D=784, H=500, Z=20)
    x = O.synthetic_mnist(n=2000)
    order = np.random.default_rng(3).permutation(20).astype(np.int32)
    outs = []
    for eager in (True, False):
        ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, 100, max_eval_rows=500)
        ctx.comm_init(_lib.Context.comm_unique_id(), 0, 1)
        ctx.set_data(x)
        ctx.set_params(O.flatten(O.init_params(cfg)))
        ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
        ctx.set_step(0)
        if eager:
            for i in order:
                ctx.update(int(i))
        else:
            ctx.update_many(order)
        s, n = ctx.epoch_elbo()
        outs.append((s, n, ctx.get_params(), ctx.get_adagrad_state()))
        ctx.close()
    assert outs[0][:2] == outs[1][:2]
    assert np.array_equal(outs[0][2], outs[1][2]) and np.array_equal(outs[0][3], outs[1][3])
