"""Optimizer plug-in mirror of /root/reference/degenerate-vae/infalg.py.

The reference's contract (infalg.py:9-41): an `InferenceAlgorithm` has `name()`,
`construct(f, theta) -> updates` (a list of (shared, new value) pairs that Theano applies
simultaneously after evaluating f) and `getinputs()` (the extra run-time inputs).
`AdaGrad.construct` (infalg.py:148-164) appends, per parameter, a fresh zero accumulator
g_ac with the pair (g_ac, g_ac + g^2) and the pair (theta, theta + eta*g/(sqrt(g_ac') + 1e-6)).

Here the arithmetic of those pairs runs inside the HIP kernels (fused into the
weight-gradient epilogues of libvaeb_hip.so, over one flat accumulator arena), so
`construct` returns the same list shape with symbolic right-hand sides -- `AccumulateSq`
and `AdaGradStep` records naming the parameter, eta and eps -- and the objective the list
is built for (`f`: a `VAEB` / `VAE` model or the AE engine) BINDS it: it checks that the
pairs cover each of its parameters exactly once with one (eta, eps), that the pairs are the
engine's own accumulators and parameters, and takes eta as its learning rate.  The
accumulator of the pair is a live view of the engine's arena (`get_value` / `set_value`),
the object Theano's `shared(np.zeros(...))` was.  The same rule is VAEB.getUpdates
(VAEB.py:426-444); only AdaGrad is on the hot path: the reference's
AdaDelta / GradientAscent / HMC are not provided (Appendix B: AdaDelta's rho setter is
broken, GradientAscent and HMC are unfinished), and `bind_updates` rejects any other rule.
"""
from __future__ import annotations

import abc
from typing import NamedTuple

import numpy as np

ADAGRAD_EPS = 1e-6   # infalg.py:158


class AccumulateSq(NamedTuple):
    """Right-hand side g_ac + T.sqr(T.grad(f, theta)) (infalg.py:157)."""
    param: object


class AdaGradStep(NamedTuple):
    """Right-hand side theta + eta * g / (T.sqrt(g_ac_new) + eps) (infalg.py:158)."""
    param: object
    accumulator: object
    eta: float
    eps: float


class Accumulator:
    """The g_ac shared variable of one parameter (infalg.py:153): a view of the engine's
    Adagrad arena.  `owner` provides `_acc_slice(param) -> (get, set)`."""

    def __init__(self, owner, param):
        self._owner, self.param = owner, param
        self.name = "g_ac_" + str(getattr(param, "name", "theta"))

    def get_value(self, borrow=False):
        return self._owner._acc_get(self.param)

    def set_value(self, value, borrow=False):
        self._owner._acc_set(self.param, np.asarray(value, np.float32))

    def __repr__(self):
        return f"Accumulator({self.name})"


class InferenceAlgorithm(abc.ABC):
    """infalg.py:9-41."""

    @abc.abstractmethod
    def name(self) -> str: ...

    @abc.abstractmethod
    def construct(self, f, theta) -> list: ...

    @abc.abstractmethod
    def getinputs(self) -> list: ...


class AdaGrad(InferenceAlgorithm):
    """infalg.py:141-183."""

    def __init__(self, eta):
        self.eta = eta

    def name(self):
        return "AdaGrad"

    def construct(self, f, theta):
        """infalg.py:148-164: per parameter, (g_ac, g_ac + g^2) then (theta, theta + dx).
        `f` is the objective's owner (it holds the accumulator arena)."""
        updates = []
        for t in theta:
            g_ac = Accumulator(f, t)
            updates.append((g_ac, AccumulateSq(t)))
            updates.append((t, AdaGradStep(t, g_ac, self.eta, ADAGRAD_EPS)))
        return updates

    def getinputs(self):
        return []

    @property
    def eta(self):
        return self._eta

    @eta.setter
    def eta(self, eta):
        if not eta > 0:
            raise ValueError("eta must be greater than zero and less than one.")   # infalg.py:174-176
        self._eta = float(eta)

    def rule(self):
        """The update the kernels apply, as (eta, eps)."""
        return self._eta, ADAGRAD_EPS


def bind_updates(owner, params, updates):
    """What an engine does with `construct`'s list: check that it is the fused AdaGrad rule
    over exactly `params` (each once, with its own accumulator of `owner`) and return
    (eta, eps).  Anything else -- another rule, a foreign parameter, a missing or repeated
    pair, mixed learning rates -- raises, since the kernels apply only that rule."""
    ids = {id(p): p for p in params}
    acc_seen, step_seen, rates = set(), set(), set()
    for lhs, rhs in updates:
        if isinstance(rhs, AccumulateSq):
            if not isinstance(lhs, Accumulator) or lhs._owner is not owner or lhs.param is not rhs.param:
                raise ValueError(f"accumulator pair {lhs!r} does not belong to this engine")
            key, seen = id(rhs.param), acc_seen
        elif isinstance(rhs, AdaGradStep):
            if lhs is not rhs.param or rhs.accumulator._owner is not owner:
                raise ValueError(f"update pair for {lhs!r} does not step that parameter")
            key, seen = id(rhs.param), step_seen
            rates.add((rhs.eta, rhs.eps))
        else:
            raise NotImplementedError(f"the HIP engines apply the AdaGrad rule only, not {type(rhs).__name__}")
        if key not in ids:
            raise ValueError(f"update targets a parameter this engine does not own: {rhs.param!r}")
        if key in seen:
            raise ValueError(f"parameter {rhs.param!r} updated twice")
        seen.add(key)
    if acc_seen != set(ids) or step_seen != set(ids):
        raise ValueError("updates must cover every parameter once (accumulator and step)")
    if len(rates) != 1:
        raise ValueError(f"one (eta, eps) per engine, got {sorted(rates)}")
    return rates.pop()
