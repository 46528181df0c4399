"""Host mirror of /root/reference/degenerate-vae/ae.py over the HIP autoencoder engine.

`ConstructAE(Xtr, Denc, Dz, Ddec, f, s2, inf, otype)` keeps the reference's signature and
returns the same five things (ae.py:41-117): `train(idx)` (one AdaGrad step on the rows
Xtr[idx], returning loglik / len(idx)), `reconstruct(X)`, `encode(X)`, `decode(Z)` and
`theta`, a list of parameters with `get_value()` / `set_value()` in the reference order.
All compute runs in libvaeb_hip.so (vaeb_ae_*, vaeb_amd/csrc/ae_mlp.hpp); there is no CPU
fallback.  Initialisation draws every weight and bias from the GLOBAL numpy RNG in the
reference's construction order (mlp.py:36-49), so `numpy.random.seed(s)` before
ConstructAE reproduces the reference's theta_0.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .infalg import AdaGrad, bind_updates

_ACT_NAMES = {"tanh": "tanh", "sigmoid": "sigmoid", "logistic": "sigmoid", "relu": "relu"}


def _act_name(f):
    key = f if isinstance(f, str) else getattr(f, "__name__", str(f))
    key = key.split(".")[-1].lower()
    if key not in _ACT_NAMES:
        raise ValueError(f"activation {f!r} not supported (tanh | sigmoid | relu)")
    return _ACT_NAMES[key]


def _values(X):
    return np.asarray(X.get_value() if hasattr(X, "get_value") else X, np.float32)


def param_shapes(Dobs, Denc, Dz, Ddec, otype):
    """theta order of ae.py:51,56,64,72."""
    d_in = [Dobs] + list(Denc)
    shp = [(f"W{i}", (d_in[i], d_in[i + 1])) for i in range(len(Denc))]
    shp += [(f"b{i}", (Denc[i],)) for i in range(len(Denc))]
    shp += [("Wz", (Denc[-1], Dz)), ("bz", (Dz,))]
    d_dec = [Dz] + list(Ddec)
    shp += [(f"W{i}", (d_dec[i], d_dec[i + 1])) for i in range(len(Ddec))]
    shp += [(f"b{i}", (Ddec[i],)) for i in range(len(Ddec))]
    if otype == "binary":
        shp += [("Wout", (Ddec[-1], Dobs)), ("bout", (Dobs,))]
    else:
        shp += [("Wmu", (Ddec[-1], Dobs)), ("Wlogs2", (Ddec[-1], Dobs)), ("bmu", (Dobs,)), ("blogs2", (Dobs,))]
    return shp


class SharedParam:
    """A slice of the device parameter arena with the Theano shared-variable accessors."""

    def __init__(self, ctx, name, shape, offset):
        self.ctx, self.name, self.shape, self.offset = ctx, name, shape, offset
        self.size = int(np.prod(shape))

    def get_value(self):
        return self.ctx.get_params()[self.offset:self.offset + self.size].reshape(self.shape).copy()

    def set_value(self, v):
        flat = self.ctx.get_params()
        flat[self.offset:self.offset + self.size] = np.asarray(v, np.float32).ravel()
        self.ctx.set_params(flat)

    def __repr__(self):
        return f"SharedParam({self.name}, {self.shape})"


class _AccArena:
    """Owner of the AdaGrad accumulators `inf.construct` hands out (views of the engine's
    accumulator arena, one slice per SharedParam)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def _acc_get(self, p):
        return self.ctx.get_adagrad_state()[p.offset:p.offset + p.size].reshape(p.shape).copy()

    def _acc_set(self, p, value):
        flat = self.ctx.get_adagrad_state()
        flat[p.offset:p.offset + p.size] = value.ravel()
        self.ctx.set_adagrad_state(flat)


def ConstructAE(Xtr, Denc=(500,), Dz=20, Ddec=(500,), f="tanh", s2=1.0, inf=None, otype="binary",
                max_batch=None, device=0):
    """ae.py:41-117.  Returns (train, reconstruct, encode, decode, theta)."""
    if otype not in ("binary", "cont"):
        raise ValueError("otype currently only supports binary.")   # ae.py:74-75 (and cont)
    inf = inf if inf is not None else AdaGrad(0.01)
    Xtr = _values(Xtr)
    Denc, Ddec = list(Denc), list(Ddec)
    Dobs = Xtr.shape[1]
    shapes = param_shapes(Dobs, Denc, Dz, Ddec, otype)
    # mlp.WeightMatrix / BiasVector: N(0, 0.01) from the global RNG, construction order
    theta0 = [np.random.normal(0.0, 0.01, size=s).astype(np.float32) for _, s in shapes]
    mb = int(max_batch) if max_batch else max(100, min(4096, Xtr.shape[0]))
    ctx = _lib.AEContext(Dobs, Denc, Dz, Ddec, otype=otype, act=_act_name(f), s2=s2, eta=inf.eta, max_batch=mb,
                         device=device)
    ctx.set_data(Xtr)
    ctx.set_params(np.concatenate([t.ravel() for t in theta0]))
    offs = np.cumsum([0] + [int(np.prod(s)) for _, s in shapes])
    theta = [SharedParam(ctx, n, s, int(o)) for (n, s), o in zip(shapes, offs[:-1])]
    # ae.py:80: updates = inf.construct(logjoint, theta), bound to the engine's fused rule
    arena = _AccArena(ctx)
    updates = inf.construct(arena, theta)
    bind_updates(arena, theta, updates)

    def train(idx):
        return ctx.train(np.asarray(idx, np.int32))

    train.ctx = ctx
    return train, ctx.reconstruct, ctx.encode, ctx.decode, theta


def rmse(X, Xpr):
    """ae.py:121-122."""
    return float(np.sqrt(np.mean(np.sum((X - Xpr) ** 2, 1))))


def train_epochs(train, Ntr, epochs, batch_size=100, verbose=True):
    """The LearnMNIST / LearnFreyFace loop (ae.py:140-151, 179-190): a fresh global-RNG
    permutation per epoch, batches of batch_size with the last partial batch kept.  The
    whole epoch is enqueued with one host sync (vaeb_ae_train_many)."""
    loglik = []
    for i in range(epochs):
        idx = np.random.permutation(np.arange(Ntr)).astype(np.int32)
        loglik.extend(train.ctx.train_many(idx, batch_size).tolist())
        if verbose:
            print("Epoch " + str(i) + ". mean loglik = " + str(loglik[-1]))
    return loglik


def LearnAE(Xtr, Xte, epochs, Dz, hidden, otype, batch_size=100, verbose=True):
    """Shared body of LearnFreyFace (ae.py:130-162) / LearnMNIST (ae.py:169-201), minus the
    matplotlib learning-curve file; returns (reconstruct, encode, decode, loglik, rmse_tr, rmse_te)."""
    train, reconstruct, encode, decode, theta = ConstructAE(Xtr, Denc=[hidden], Dz=Dz, Ddec=[hidden], otype=otype,
                                                            inf=AdaGrad(0.01))
    if verbose:
        print("Training the autoencoder.")
    loglik = train_epochs(train, Xtr.shape[0], epochs, batch_size, verbose)
    rtr, rte = rmse(Xtr, reconstruct(Xtr)), rmse(Xte, reconstruct(Xte))
    if verbose:
        print("training rmse = " + str(rtr))
        print("testing rmse = " + str(rte))
    return reconstruct, encode, decode, loglik, rtr, rte
