"""Optimizer plug-in mirror of /root/reference/degenerate-vae/infalg.py.

The reference's `InferenceAlgorithm.construct(f, theta)` builds Theano update pairs; here
the rule itself runs inside the HIP kernels (fused into the weight-gradient epilogues of
libvaeb_hip.so), so an inference object is the configuration the engines read:
`AdaGrad(eta)` -> g_ac += g^2; theta += eta * g / (sqrt(g_ac) + 1e-6) (infalg.py:148-164),
the same rule as VAEB.getUpdates (VAEB.py:426-444).  Only AdaGrad is on the hot path
(SURVEY 8(a) A16); the reference's AdaDelta / GradientAscent / HMC are not ported
(Appendix B: AdaDelta's rho setter is broken, GradientAscent and HMC are unfinished).
"""
from __future__ import annotations

import abc

ADAGRAD_EPS = 1e-6   # infalg.py:158


class InferenceAlgorithm(abc.ABC):
    """infalg.py:9-41: an optimizer exposes a name and the hyper-parameters the engine uses."""

    @abc.abstractmethod
    def name(self) -> str: ...

    @abc.abstractmethod
    def getinputs(self) -> list: ...


class AdaGrad(InferenceAlgorithm):
    """infalg.py:141-183."""

    def __init__(self, eta):
        self.eta = eta

    def name(self):
        return "AdaGrad"

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
