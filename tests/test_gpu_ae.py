"""Parity of the degenerate-vae autoencoder engine (vaeb_ae_*, vaeb_amd/csrc/ae_mlp.hpp)
against the CPU oracle (oracle/ae_oracle.py, float64) on identical theta / acc / rows.

Tolerances (fp32 MFMA, ~1-ulp hardware transcendentals):
  * train's value (loglik / n): relative <= 2e-5
  * theta' after AdaGrad: |diff| <= 1e-3 * eta for all but a 1e-4 fraction of elements
    (the first step is ~eta * sign(g)), never more than 2 * eta; accumulator relative <= 1e-4
  * encode / decode / reconstruct: absolute <= 2e-5
  * 8-step epoch (gathered permutation, last partial batch kept): per-step relative <= 1e-4
"""
import numpy as np
import pytest

from oracle import ae_oracle as A

pytestmark = pytest.mark.gpu

CASES = [
    ("mnist_like", dict(Dobs=784, Denc=(64,), Dz=8, Ddec=(64,), otype="binary"), 50),
    ("frey_like_cont", dict(Dobs=560, Denc=(48,), Dz=6, Ddec=(40,), otype="cont"), 40),
    ("deep_odd", dict(Dobs=37, Denc=(29, 17), Dz=5, Ddec=(13, 21), otype="binary", s2=2.0), 23),
    ("deep_cont_sigmoid", dict(Dobs=48, Denc=(20,), Dz=4, Ddec=(18, 11), otype="cont", act="sigmoid"), 30),
    ("relu", dict(Dobs=64, Denc=(32,), Dz=8, Ddec=(32,), otype="binary", act="relu"), 32),
]


def data_for(cfg, n, seed=0):
    rng = np.random.default_rng(seed)
    if cfg.otype == "binary":
        return (rng.random((n, cfg.Dobs)) < 0.3).astype(np.float32)
    return rng.beta(2.0, 2.0, size=(n, cfg.Dobs)).astype(np.float32)


def make_ctx(cfg, max_batch):
    from vaeb_amd import _lib
    return _lib.AEContext(cfg.Dobs, cfg.Denc, cfg.Dz, cfg.Ddec, otype=cfg.otype, act=cfg.act, s2=cfg.s2,
                          eta=cfg.eta, max_batch=max_batch)


def check_theta(new, ref, eta):
    d = np.abs(new - ref)
    assert d.max() <= 2 * eta + 1e-7, d.max()
    assert float((d > 1e-3 * eta).mean()) <= 1e-4


@pytest.mark.parametrize("name,kw,B", CASES, ids=[c[0] for c in CASES])
def test_ae_train_step_parity(name, kw, B):
    cfg = A.AEConfig(**kw)
    X = data_for(cfg, 4 * B)
    params = A.init_params(cfg)
    rng = np.random.default_rng(2)
    acc = [np.full(p.shape, 1e-4, np.float32) for p in params]
    idx = rng.choice(X.shape[0], size=B, replace=False).astype(np.int32)   # Xtr[idx] gather
    ctx = make_ctx(cfg, B)
    ctx.set_data(X)
    ctx.set_params(A.flatten(params))
    ctx.set_adagrad_state(A.flatten(acc))
    got = ctx.train(idx)
    p64 = [p.astype(np.float64) for p in params]
    a64 = [a.astype(np.float64) for a in acc]
    ref, ref_p, ref_a, aux = A.train_step(p64, a64, X.astype(np.float64), idx, cfg)
    assert abs(got - ref) <= 2e-5 * abs(ref), (got, ref)
    check_theta(ctx.get_params(), A.flatten(ref_p), cfg.eta)
    na, ra = ctx.get_adagrad_state(), A.flatten(ref_a)
    assert np.linalg.norm(na - ra) <= 1e-4 * np.linalg.norm(ra)
    ctx.close()


@pytest.mark.parametrize("name,kw,B", CASES[:3], ids=[c[0] for c in CASES[:3]])
def test_ae_predict_parity(name, kw, B):
    cfg = A.AEConfig(**kw)
    X = data_for(cfg, 3 * B, seed=4)
    params = A.init_params(cfg, seed=7)
    params = [(p * 30).astype(np.float32) for p in params]   # non-trivial activations
    ctx = make_ctx(cfg, B)
    ctx.set_data(X)
    ctx.set_params(A.flatten(params))
    p64 = [p.astype(np.float64) for p in params]
    out = A.forward_backward(p64, X.astype(np.float64), cfg, need_grad=False)
    assert np.abs(ctx.reconstruct(X) - out["Xpr"]).max() <= 2e-5
    z = ctx.encode(X)
    assert np.abs(z - out["Z"]).max() <= 2e-5 * max(1.0, np.abs(out["Z"]).max())
    dec = ctx.decode(out["Z"].astype(np.float32))
    assert np.abs(dec - out["Xpr"]).max() <= 2e-5
    ctx.close()


def test_ae_epoch_with_partial_batch_tracks_oracle():
    cfg = A.AEConfig(Dobs=96, Denc=(40,), Dz=6, Ddec=(40,), otype="binary")
    Ntr, B = 350, 100
    X = data_for(cfg, Ntr, seed=9)
    params = A.init_params(cfg)
    ctx = make_ctx(cfg, B)
    ctx.set_data(X)
    ctx.set_params(A.flatten(params))
    rs = np.random.RandomState(15485863)
    batches = A.epoch_batches(Ntr, B, rs) + A.epoch_batches(Ntr, B, rs)   # two epochs, 4 + 4 steps
    got = list(ctx.train_many(np.concatenate(batches[:4]), B)) + list(ctx.train_many(np.concatenate(batches[4:]), B))
    p = [q.astype(np.float64) for q in params]
    a = [np.zeros_like(q) for q in p]
    ref = []
    for b in batches:
        v, p, a, _ = A.train_step(p, a, X.astype(np.float64), b, cfg)
        ref.append(v)
    assert [len(b) for b in batches[:4]] == [100, 100, 100, 50]
    for g, r in zip(got, ref):
        assert abs(g - r) <= 1e-4 * abs(r), (g, r)
    d = np.abs(ctx.get_params() - A.flatten(p))
    assert float((d > 1e-2 * cfg.eta).mean()) <= 1e-3
    ctx.close()


def test_construct_ae_mirror_learns():
    """vaeb_amd.ae.ConstructAE keeps the reference's API (ae.py:41-117) and its theta_0
    follows the global numpy RNG draws; a few epochs raise the log-likelihood."""
    from vaeb_amd import ae
    cfg = A.AEConfig(Dobs=784, Denc=(500,), Dz=5, Ddec=(500,), otype="binary")
    X = data_for(cfg, 1000, seed=3)
    np.random.seed(15485863)
    train, reconstruct, encode, decode, theta = ae.ConstructAE(X, Denc=[500], Dz=5, Ddec=[500])
    ref0 = A.init_params(cfg, seed=15485863)
    assert all(np.array_equal(t.get_value(), r) for t, r in zip(theta, ref0))
    ll = ae.train_epochs(train, X.shape[0], 3, verbose=False)
    assert len(ll) == 30 and np.isfinite(ll).all() and ll[-1] > ll[0]
    assert ae.rmse(X, reconstruct(X)) < ae.rmse(X, np.zeros_like(X))
    z = encode(X[:7])
    assert z.shape == (7, 5) and decode(z).shape == (7, 784)
