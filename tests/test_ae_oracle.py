"""The degenerate-vae autoencoder oracle (oracle/ae_oracle.py) against float64 torch
autograd of the same logjoint (ae.py:77-78), and its init / epoch-batching conventions."""
import numpy as np
import pytest
import torch

from oracle import ae_oracle as A

CASES = [
    dict(Dobs=30, Denc=(12,), Dz=4, Ddec=(11,), otype="binary"),
    dict(Dobs=24, Denc=(10, 7), Dz=3, Ddec=(6, 9), otype="binary", s2=2.0),
    dict(Dobs=20, Denc=(9,), Dz=5, Ddec=(8,), otype="cont"),
    dict(Dobs=16, Denc=(8, 6), Dz=2, Ddec=(7,), otype="cont", act="sigmoid"),
]


def torch_logjoint(params, X, cfg):
    names = [n for n, _ in A.param_shapes(cfg)]
    p = dict(zip(names, params))
    f = {"tanh": torch.tanh, "sigmoid": torch.sigmoid, "relu": torch.relu}[cfg.act]
    H = X
    for i in range(len(cfg.Denc)):
        H = f(H @ p[f"Wenc{i}"] + p[f"benc{i}"])
    Z = H @ p["Wz"] + p["bz"]
    G = Z
    for i in range(len(cfg.Ddec)):
        G = f(G @ p[f"Wdec{i}"] + p[f"bdec{i}"])
    if cfg.otype == "binary":
        P = torch.sigmoid(G @ p["Wout"] + p["bout"])
        ll = (X * torch.log(P + 1e-7) + (1 - X) * torch.log(1 - P + 1e-7)).sum()
    else:
        mu = torch.sigmoid(G @ p["Wmu"] + p["bmu"])
        ls2 = G @ p["Wlogs2"] + p["blogs2"]
        ll = -0.5 * (np.log(2 * np.pi) + ls2 + (X - mu) ** 2 / torch.exp(ls2)).sum()
    lp = -0.5 * sum(((q ** 2) / cfg.s2 + np.log(2 * np.pi * cfg.s2)).sum() for q in params)
    lz = -0.5 * (Z ** 2 + np.log(2 * np.pi)).sum()
    return ll, ll + lp + lz


@pytest.mark.parametrize("kw", CASES)
def test_ae_gradient_matches_autograd(kw):
    cfg = A.AEConfig(**kw)
    rng = np.random.default_rng(0)
    params = [(0.3 * rng.standard_normal(s)).astype(np.float64) for _, s in A.param_shapes(cfg)]
    X = rng.random((7, cfg.Dobs))
    if cfg.otype == "binary":
        X = (X < 0.4).astype(np.float64)
    out = A.forward_backward(params, X, cfg)
    tp = [torch.tensor(q, requires_grad=True) for q in params]
    ll, lj = torch_logjoint(tp, torch.tensor(X), cfg)
    lj.backward()
    assert abs(out["loglik"] - ll.item()) <= 1e-10 * max(1.0, abs(ll.item()))
    assert abs(out["logjoint"] - lj.item()) <= 1e-10 * max(1.0, abs(lj.item()))
    for g, t in zip(out["grads"], tp):
        assert np.allclose(g, t.grad.numpy(), rtol=1e-9, atol=1e-11)


def test_init_order_and_shapes():
    cfg = A.AEConfig(Dobs=784, Denc=(500,), Dz=5, Ddec=(500,))
    ps = A.init_params(cfg)
    assert [p.shape for p in ps] == [s for _, s in A.param_shapes(cfg)]
    rs = np.random.RandomState(15485863)
    w0 = rs.normal(0.0, 0.01, size=(784, 500)).astype(np.float32)
    b0 = rs.normal(0.0, 0.01, size=(500,)).astype(np.float32)
    assert np.array_equal(ps[0], w0) and np.array_equal(ps[1], b0)   # Wenc0 then benc0 (ae.py:48)
    assert all(float(np.std(p)) > 0 for p in ps)                      # biases are drawn too (mlp.py:39)


def test_epoch_batches_keep_last_partial_batch():
    rs = np.random.RandomState(1)
    b = A.epoch_batches(250, 100, rs)
    assert [len(x) for x in b] == [100, 100, 50]
    assert sorted(np.concatenate(b).tolist()) == list(range(250))
