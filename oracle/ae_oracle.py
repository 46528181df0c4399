"""CPU oracle for the degenerate-vae deterministic autoencoder step -- TEST INFRASTRUCTURE ONLY.

NumPy restatement of /root/reference/degenerate-vae (Python 2 + Theano, not runnable
here) used to CHECK the HIP layer-stack engine (vaeb_amd/csrc/ae_mlp.hpp); the product
path never imports it.

  * ae.py:41-117 ConstructAE: encoder MLP (mlp.py:66-74 ConstructMLP, f = tanh), linear
    latent Z = Hz Wz + bz (ae.py:49), decoder MLP, output layer by otype (ae.py:58-73),
    logjoint = loglik + NormalPrior(theta, s2) + NormalPrior([Z], 1) (ae.py:77-78),
    train(idx) returns loglik / |idx| over the gathered rows Xtr[idx] (ae.py:82-89).
  * mlp.py:36-49 WeightMatrix / BiasVector: N(0, 0.01) draws (std 0.01) from the GLOBAL
    numpy RandomState, in construction order; mlp.py:87-91 ConstructNormalPrior.
  * logpdf.py:46-47 OutToProbs (sigmoid), :72-73 OutToReal, :85-86 bernoulli with the
    1e-7 inside both logs, :112-114 indep_normal.
  * infalg.py:148-164 AdaGrad.construct: g = dlogjoint/dtheta; g_ac += g^2;
    theta += eta g / (sqrt(g_ac) + 1e-6).

Pinning: the logpdf.py:119-123 known answer (tests/test_oracle_pins.py); the gradient of
this restatement is checked against float64 torch autograd (tests/test_ae_oracle.py).
Bitwise Theano behaviour is "parity unpinned" (see DESIGN.md).
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

LOG2PI = math.log(2.0 * math.pi)
EPS_LOG = 1e-7   # logpdf.py:86


@dataclasses.dataclass
class AEConfig:
    Dobs: int
    Denc: tuple = (500,)
    Dz: int = 20
    Ddec: tuple = (500,)
    otype: str = "binary"      # "binary" | "cont" (ae.py:58-73)
    s2: float = 1.0            # prior variance on theta (ae.py:41)
    eta: float = 0.01          # AdaGrad(0.01)
    act: str = "tanh"          # f (ae.py:41)


def param_shapes(cfg: AEConfig):
    """theta order (ae.py:51,56,64,72): Wenc..., benc..., Wz, bz, Wdec..., bdec..., then
    [Wout, bout] (binary) or [Wmu, Wlogs2, bmu, blogs2] (cont)."""
    denc, ddec = list(cfg.Denc), list(cfg.Ddec)
    d_in = [cfg.Dobs] + denc
    shp = [(f"Wenc{i}", (d_in[i], d_in[i + 1])) for i in range(len(denc))]
    shp += [(f"benc{i}", (denc[i],)) for i in range(len(denc))]
    shp += [("Wz", (denc[-1], cfg.Dz)), ("bz", (cfg.Dz,))]
    d_dec = [cfg.Dz] + ddec
    shp += [(f"Wdec{i}", (d_dec[i], d_dec[i + 1])) for i in range(len(ddec))]
    shp += [(f"bdec{i}", (ddec[i],)) for i in range(len(ddec))]
    if cfg.otype == "binary":
        shp += [("Wout", (ddec[-1], cfg.Dobs)), ("bout", (cfg.Dobs,))]
    else:
        shp += [("Wmu", (ddec[-1], cfg.Dobs)), ("Wlogs2", (ddec[-1], cfg.Dobs)),
                ("bmu", (cfg.Dobs,)), ("blogs2", (cfg.Dobs,))]
    return shp


def init_params(cfg: AEConfig, seed=15485863):
    """Draws in construction order from numpy's global-style RandomState (ae.py:48-72):
    every weight AND bias ~ N(0, 0.01) (mlp.py:39,49), float32."""
    rs = np.random.RandomState(seed)
    denc, ddec = list(cfg.Denc), list(cfg.Ddec)
    d_in = [cfg.Dobs] + denc
    draws = {}
    for i in range(len(denc)):                       # mlp.WeightMatrices([Dobs] + Denc)
        draws[f"Wenc{i}"] = rs.normal(0.0, 0.01, size=(d_in[i], d_in[i + 1]))
    for i in range(len(denc)):                       # mlp.BiasVectors(Denc)
        draws[f"benc{i}"] = rs.normal(0.0, 0.01, size=(denc[i],))
    draws["Wz"] = rs.normal(0.0, 0.01, size=(denc[-1], cfg.Dz))
    draws["bz"] = rs.normal(0.0, 0.01, size=(cfg.Dz,))
    d_dec = [cfg.Dz] + ddec
    for i in range(len(ddec)):
        draws[f"Wdec{i}"] = rs.normal(0.0, 0.01, size=(d_dec[i], d_dec[i + 1]))
    for i in range(len(ddec)):
        draws[f"bdec{i}"] = rs.normal(0.0, 0.01, size=(ddec[i],))
    if cfg.otype == "binary":
        draws["Wout"] = rs.normal(0.0, 0.01, size=(ddec[-1], cfg.Dobs))
        draws["bout"] = rs.normal(0.0, 0.01, size=(cfg.Dobs,))
    else:
        draws["Wmu"] = rs.normal(0.0, 0.01, size=(ddec[-1], cfg.Dobs))
        draws["Wlogs2"] = rs.normal(0.0, 0.01, size=(ddec[-1], cfg.Dobs))
        draws["bmu"] = rs.normal(0.0, 0.01, size=(cfg.Dobs,))
        draws["blogs2"] = rs.normal(0.0, 0.01, size=(cfg.Dobs,))
    return [draws[n].astype(np.float32) for n, _ in param_shapes(cfg)]


def flatten(params):
    return np.concatenate([np.asarray(p, np.float32).ravel() for p in params])


def unflatten(flat, cfg: AEConfig):
    out, o = [], 0
    for _, s in param_shapes(cfg):
        n = int(np.prod(s))
        out.append(np.asarray(flat[o:o + n]).reshape(s))
        o += n
    return out


def _act(name, a):
    if name == "tanh":
        return np.tanh(a)
    if name == "sigmoid":
        return 1.0 / (1.0 + np.exp(-a))
    if name == "relu":
        return np.maximum(a, 0.0)
    raise ValueError(name)


def _dact(name, h):
    """Derivative in terms of the activation output h."""
    if name == "tanh":
        return 1.0 - h * h
    if name == "sigmoid":
        return h * (1.0 - h)
    if name == "relu":
        return (h > 0).astype(h.dtype)
    raise ValueError(name)


def forward_backward(params, X, cfg: AEConfig, need_grad=True):
    """One evaluation of the ConstructAE graph on rows X (already gathered) and the
    reverse-mode gradient of logjoint (ae.py:77-78) in theta order."""
    names = [n for n, _ in param_shapes(cfg)]
    p = dict(zip(names, params))
    dt = params[0].dtype
    X = np.asarray(X, dt)
    ne, nd = len(cfg.Denc), len(cfg.Ddec)
    H = [X]
    for i in range(ne):
        H.append(_act(cfg.act, H[-1] @ p[f"Wenc{i}"] + p[f"benc{i}"]))
    Z = H[-1] @ p["Wz"] + p["bz"]
    G = [Z]
    for i in range(nd):
        G.append(_act(cfg.act, G[-1] @ p[f"Wdec{i}"] + p[f"bdec{i}"]))
    out = dict(H=H, Z=Z, G=G)
    if cfg.otype == "binary":
        a = G[-1] @ p["Wout"] + p["bout"]
        P = 1.0 / (1.0 + np.exp(-a))
        loglik = float((X * np.log(P + EPS_LOG) + (1 - X) * np.log(1.0 - P + EPS_LOG)).sum(dtype=np.float64))
        out["Xpr"] = P
    else:
        amu = G[-1] @ p["Wmu"] + p["bmu"]
        mu = 1.0 / (1.0 + np.exp(-amu))
        ls2 = G[-1] @ p["Wlogs2"] + p["blogs2"]
        r = X - mu
        loglik = float((-0.5 * (LOG2PI + ls2 + r * r / np.exp(ls2))).sum(dtype=np.float64))
        out["Xpr"] = mu
    out["loglik"] = loglik
    s2 = cfg.s2
    logprior = -0.5 * sum(float((q.astype(np.float64) ** 2 / s2 + math.log(2 * math.pi * s2)).sum()) for q in params)
    zprior = -0.5 * float((Z.astype(np.float64) ** 2 + LOG2PI).sum())
    out["logjoint"] = loglik + logprior + zprior
    if not need_grad:
        return out

    g = {}
    if cfg.otype == "binary":
        dP = X / (P + EPS_LOG) - (1 - X) / (1.0 - P + EPS_LOG)
        dA = dP * P * (1 - P)
        g["Wout"] = G[-1].T @ dA
        g["bout"] = dA.sum(0)
        dG = dA @ p["Wout"].T
    else:
        e = np.exp(-ls2)
        dAmu = r * e * mu * (1 - mu)
        dAls = -0.5 + 0.5 * r * r * e
        g["Wmu"] = G[-1].T @ dAmu
        g["bmu"] = dAmu.sum(0)
        g["Wlogs2"] = G[-1].T @ dAls
        g["blogs2"] = dAls.sum(0)
        dG = dAmu @ p["Wmu"].T + dAls @ p["Wlogs2"].T
    for i in reversed(range(nd)):
        dPre = dG * _dact(cfg.act, G[i + 1])
        g[f"Wdec{i}"] = G[i].T @ dPre
        g[f"bdec{i}"] = dPre.sum(0)
        dG = dPre @ p[f"Wdec{i}"].T
    dZ = dG - Z                                        # + d/dZ of NormalPrior([Z], 1)
    g["Wz"] = H[-1].T @ dZ
    g["bz"] = dZ.sum(0)
    dH = dZ @ p["Wz"].T
    for i in reversed(range(ne)):
        dPre = dH * _dact(cfg.act, H[i + 1])
        g[f"Wenc{i}"] = H[i].T @ dPre
        g[f"benc{i}"] = dPre.sum(0)
        if i > 0:
            dH = dPre @ p[f"Wenc{i}"].T
    out["data_grads"] = [g[n].astype(dt) for n in names]
    out["grads"] = [(g[n] - p[n] / s2).astype(dt) for n in names]
    return out


def adagrad(params, acc, grads, eta):
    """infalg.py:148-164."""
    new_p, new_a = [], []
    for th, a, g in zip(params, acc, grads):
        a2 = a + g * g
        new_p.append((th + eta * g / (np.sqrt(a2) + 1e-6)).astype(th.dtype))
        new_a.append(a2.astype(th.dtype))
    return new_p, new_a


def train_step(params, acc, Xtr, idx, cfg: AEConfig):
    """train(idx) (ae.py:82-89): returns (loglik / |idx|, theta', acc', aux)."""
    X = Xtr[np.asarray(idx)]
    out = forward_backward(params, X, cfg)
    new_p, new_a = adagrad(params, acc, out["grads"], cfg.eta)
    return out["loglik"] / X.shape[0], new_p, new_a, out


def epoch_batches(Ntr, batch_size, rs):
    """LearnMNIST / LearnFreyFace epoch loop (ae.py:140-151): a fresh permutation per epoch,
    batches of batch_size with the last partial batch KEPT."""
    idx = rs.permutation(np.arange(Ntr)).astype(np.int32)
    return [idx[lb:min(lb + batch_size, Ntr)] for lb in range(0, Ntr, batch_size)]


def rmse(X, Xpr):
    """ae.py:121-122."""
    return float(np.sqrt(np.mean(np.sum((X - Xpr) ** 2, 1))))
