"""The optimizer plug-in contract of degenerate-vae/infalg.py:9-41, 148-164 (host logic; the
rule's arithmetic runs in the kernels and is checked by the GPU parity tests):
`AdaGrad.construct(f, theta)` returns, per parameter, the (g_ac, g_ac + g^2) and
(theta, theta + eta*g/(sqrt(g_ac') + 1e-6)) pairs in the reference's order, and an engine
binds exactly that list."""
import numpy as np
import pytest

from vaeb_amd.infalg import (ADAGRAD_EPS, AccumulateSq, Accumulator, AdaGrad, AdaGradStep,
                             InferenceAlgorithm, bind_updates)


class _P:
    def __init__(self, name, shape):
        self.name, self.shape = name, shape


class _Owner:
    """Accumulator arena stand-in: one array per parameter."""

    def __init__(self, params):
        self.acc = {id(p): np.zeros(p.shape, np.float32) for p in params}

    def _acc_get(self, p):
        return self.acc[id(p)].copy()

    def _acc_set(self, p, v):
        self.acc[id(p)][...] = v


def _setup():
    theta = [_P("W3", (4, 3)), _P("b3", (3,))]
    return theta, _Owner(theta)


def test_construct_pairs_follow_reference_order():
    theta, own = _setup()
    ups = AdaGrad(0.05).construct(own, theta)
    assert len(ups) == 2 * len(theta)
    for i, t in enumerate(theta):
        (acc, r1), (tt, r2) = ups[2 * i], ups[2 * i + 1]
        assert isinstance(acc, Accumulator) and r1 == AccumulateSq(t)          # infalg.py:160
        assert tt is t and r2 == AdaGradStep(t, acc, 0.05, ADAGRAD_EPS)          # infalg.py:161
    assert bind_updates(own, theta, ups) == (0.05, ADAGRAD_EPS)
    assert AdaGrad(0.05).getinputs() == [] and AdaGrad(0.05).name() == "AdaGrad"
    assert issubclass(AdaGrad, InferenceAlgorithm)


def test_accumulator_is_a_view_of_the_owner_arena():
    theta, own = _setup()
    acc = AdaGrad(0.01).construct(own, theta)[0][0]
    acc.set_value(np.full((4, 3), 2.5))
    assert np.all(own.acc[id(theta[0])] == 2.5) and np.all(acc.get_value() == 2.5)


def test_eta_setter_matches_reference():
    with pytest.raises(ValueError, match="eta must be greater than zero"):
        AdaGrad(0.0)                                                             # infalg.py:174-176
    a = AdaGrad(0.1)
    a.eta = 0.2
    assert a.rule() == (0.2, ADAGRAD_EPS)


def test_bind_rejects_what_the_kernels_cannot_apply():
    theta, own = _setup()
    ups = AdaGrad(0.01).construct(own, theta)
    with pytest.raises(ValueError, match="cover every parameter"):
        bind_updates(own, theta, ups[:2])
    with pytest.raises(ValueError, match="twice"):
        bind_updates(own, theta, ups + ups[:2])
    with pytest.raises(ValueError, match="one \\(eta, eps\\)"):
        bind_updates(own, theta, ups[:2] + AdaGrad(0.02).construct(own, theta)[2:])
    with pytest.raises(ValueError, match="does not belong"):
        bind_updates(own, theta, AdaGrad(0.01).construct(_Owner(theta), theta))
    with pytest.raises(ValueError, match="does not own"):
        bind_updates(own, theta[:1], ups)
    with pytest.raises(NotImplementedError, match="AdaGrad rule only"):
        bind_updates(own, theta, [(theta[0], ("theta + eta * g",))])
