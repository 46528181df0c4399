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
