"""Cross-check the oracle's hand-written backward against float64
torch autograd of the same objective (VAEB.py:245-399), for every estimator/decoder/
objective combination the HIP path implements."""
import math

import numpy as np
import pytest
import torch

from oracle import vaeb_oracle as O


def torch_objective(params, x, eps, cfg):
    p = dict(zip(cfg.names, params))
    B = x.shape[0]
    L = eps.shape[0]
    h = torch.tanh(x @ p["W3"] + p["b3"])
    mu = h @ p["W4"] + p["b4"]
    lv = h @ p["W5"] + p["b5"]
    z = mu[None] + torch.exp(0.5 * lv)[None] * eps
    hd = torch.tanh(z.reshape(L * B, -1) @ p["W1"] + p["b1"])
    a2 = hd @ p["W2"] + p["b2"]
    xr = x.repeat(L, 1)
    if cfg.continuous:
        y = torch.sigmoid(a2)
        a6 = hd @ p["W6"] + p["b6"]
        logp = (-0.5 * math.log(2 * math.pi) - 0.5 * a6 - 0.5 * (xr - y) ** 2 / torch.exp(a6)).sum(1)
    else:
        y = torch.sigmoid(a2)
        logp = (xr * torch.log(y) + (1 - xr) * torch.log(1 - y)).sum(1)
    logp = logp.reshape(L, B)
    if cfg.estimator == "LA":
        prior = (-0.5 * math.log(2 * math.pi) - 0.5 * z ** 2).sum(2)
        logq = (-0.5 * math.log(2 * math.pi) - 0.5 * lv[None] - 0.5 * (z - mu[None]) ** 2 / torch.exp(lv)[None]).sum(2)
        sgvb = (logp + prior - logq).sum() / L
    else:
        sgvb = logp.sum() / L + (0.5 * (1 + lv - mu ** 2 - torch.exp(lv))).sum()
    if cfg.objective == "mean_map":
        return sgvb, sgvb / B
    J = sgvb
    for t in params:
        J = J - 0.5 * (t ** 2).sum()
    return sgvb, J


CASES = [
    dict(continuous=False, estimator="LB", L=1, objective="sum_prior"),
    dict(continuous=False, estimator="LB", L=3, objective="sum_prior"),
    dict(continuous=False, estimator="LA", L=2, objective="sum_prior"),
    dict(continuous=True, estimator="LB", L=1, objective="sum_prior"),
    dict(continuous=True, estimator="LA", L=2, objective="sum_prior"),
    dict(continuous=False, estimator="LB", L=1, objective="mean_map"),
    dict(continuous=True, estimator="LB", L=1, objective="mean_map"),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_backward_matches_autograd(case):
    cfg = O.Config(D=24, H=16, Z=5, **case)
    rng = np.random.default_rng(7)
    params = [(rng.standard_normal(s) * 0.3).astype(np.float64) for _, s in O.param_shapes(cfg)]
    B = 9
    x = rng.random((B, cfg.D)) if cfg.continuous else (rng.random((B, cfg.D)) < 0.3).astype(np.float64)
    eps = rng.standard_normal((cfg.L, B, cfg.Z))
    out = O.forward_backward(params, x, eps, cfg)
    tp = [torch.tensor(p, requires_grad=True) for p in params]
    sgvb, J = torch_objective(tp, torch.tensor(x), torch.tensor(eps), cfg)
    J.backward()
    assert abs(out["sgvb"] - sgvb.item()) <= 1e-10 * max(1.0, abs(sgvb.item()))
    for n, g, t in zip(cfg.names, out["grads"], tp):
        ref = t.grad.numpy()
        err = np.abs(g - ref).max()
        assert err <= 1e-10 * max(1.0, np.abs(ref).max()), (n, err)


def test_fv_gradients_closed_form():
    """g_mu = -2 mu, g_sigma = 1/sigma - 2 sigma (VAEB.py:359-363 + :392-393)."""
    mu = torch.tensor(np.random.default_rng(0).standard_normal(50), requires_grad=True)
    sig = torch.full((50,), 1e-3, dtype=torch.float64, requires_grad=True)
    J = (0.5 * (1 + torch.log(sig ** 2) - mu ** 2 - sig ** 2)).sum() - 0.5 * (mu ** 2).sum() - 0.5 * (sig ** 2).sum()
    J.backward()
    assert np.allclose(mu.grad.numpy(), -2 * mu.detach().numpy())
    s = sig.detach().numpy()
    assert np.allclose(sig.grad.numpy(), 1 / s - 2 * s)


def test_oracle_reconstruct_branches():
    """VAEB.reconstruct restatement (VAEB.py:267-300): S all-zero draws reproduce the
    z = mu branch; one draw equals the decoder at mu + exp(lv/2) eps."""
    cfg = O.Config(D=40, H=16, Z=3)
    params = [p.astype(np.float64) for p in O.init_params(cfg)]
    x = O.synthetic_mnist(n=7, D=40, seed=1).astype(np.float64)
    y0 = O.reconstruct(params, x, None, cfg)
    assert np.allclose(O.reconstruct(params, x, np.zeros((3, 7, 3)), cfg), y0, atol=1e-15)
    eps = np.random.default_rng(0).standard_normal((1, 7, 3))
    out = O.forward_backward(params, x, eps, cfg, need_grad=False)
    assert np.allclose(O.reconstruct(params, x, eps, cfg), out["y"], atol=1e-15)


@pytest.mark.parametrize("continuous", [False, True])
def test_fvs_gradients_match_autograd(continuous):
    """Weight-sampling full-variational extension (oracle fvs_step): the Adagrad step it
    takes equals the one from torch autograd of J(mu, sigma) = B (sum log p + sum KL)
    (mu + |sigma| zeta) + thetaPrior(mu, sigma) - 1/2 sum(mu^2 + sigma^2) (VAEB.py:127-129,
    349-367, 386-399)."""
    cfg = O.Config(D=12, H=6, Z=2, continuous=continuous, estimator="FV")
    rng = np.random.default_rng(11)
    B = 5
    mu = [0.3 * rng.standard_normal(s) for _, s in O.param_shapes(cfg)]
    sig = [np.full(s, 0.05) + 0.01 * rng.random(s) for _, s in O.param_shapes(cfg)]
    zeta = [rng.standard_normal(s) for _, s in O.param_shapes(cfg)]
    am = [np.zeros(s) for _, s in O.param_shapes(cfg)]
    as_ = [np.zeros(s) for _, s in O.param_shapes(cfg)]
    x = rng.random((B, cfg.D))
    if not continuous:
        x = (x < 0.5).astype(np.float64)
    eps = rng.standard_normal((1, B, cfg.Z))
    _, new_mu, new_sig, new_am, new_as, sgvb = O.fvs_step(mu, sig, am, as_, x, eps, zeta, cfg)

    tm = [torch.tensor(m, requires_grad=True) for m in mu]
    ts = [torch.tensor(s, requires_grad=True) for s in sig]
    theta = [m + torch.abs(s) * torch.tensor(z) for m, s, z in zip(tm, ts, zeta)]
    data, _ = torch_objective(theta, torch.tensor(x), torch.tensor(eps), O.Config(**{**cfg.__dict__, "estimator": "LB"}))
    tp = sum(0.5 * (1 + torch.log(s ** 2) - m ** 2 - s ** 2).sum() for m, s in zip(tm, ts))
    J = B * data + tp - 0.5 * sum((m ** 2).sum() + (s ** 2).sum() for m, s in zip(tm, ts))
    J.backward()
    assert abs(sgvb - float((B * data + tp).detach())) <= 1e-9 * abs(sgvb)
    for m, s, nm, ns, na, nb in zip(tm, ts, new_mu, new_sig, new_am, new_as):
        gm, gs = m.grad.numpy(), s.grad.numpy()
        assert np.allclose(na, gm * gm, rtol=1e-9, atol=1e-12)
        assert np.allclose(nb, gs * gs, rtol=1e-9, atol=1e-12)
        assert np.allclose(nm, m.detach().numpy() + cfg.lr * gm / (np.abs(gm) + cfg.eps), rtol=1e-9, atol=1e-12)
        assert np.allclose(ns, s.detach().numpy() + cfg.lr * gs / (np.abs(gs) + cfg.eps), rtol=1e-9, atol=1e-12)
