"""The committed golden step vectors (tests/golden/step_golden.npz, written by
tests/golden/make_step_golden.py from the float64 restatement) against the restatement as
it is now: theta0 bit-exact (RandomState(10) with the duplicated draws, VAEB.py:50-125),
intermediates / gradients / 10-step trajectories to float32 storage precision.  A change to
the oracle that moves any of them fails here before it can move a GPU parity test."""
import os

import numpy as np
import pytest

from oracle import vaeb_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "step_golden.npz")
CASES = {
    "mnist_lb": dict(D=784, H=32, Z=8),
    "frey_la_l2": dict(D=560, H=32, Z=2, continuous=True, estimator="LA", L=2),
    "mnist_mean_map": dict(D=784, H=32, Z=8, objective="mean_map"),
}


def load(name):
    with np.load(GOLD) as f:
        return {k.split("/", 1)[1]: f[k] for k in f.files if k.startswith(name + "/")}


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("name", list(CASES))
def test_restatement_reproduces_golden(name):
    g = load(name)
    cfg = O.Config(**CASES[name])
    B = int(g["B"])
    assert np.array_equal(O.flatten(O.init_params(cfg)), g["theta0"])
    p = [t.astype(np.float64) for t in O.unflatten(g["theta0"], cfg)]
    a = [np.zeros_like(t) for t in p]
    for s, b in enumerate(g["order"]):
        xb = g["x"][b * B:(b + 1) * B].astype(np.float64)
        e, p, a, aux = O.step(p, a, xb, g["eps"][s].astype(np.float64), cfg)
        assert abs(e - g["elbos"][s]) <= 1e-10 * abs(g["elbos"][s])
        if s == 0:
            for k in ("h", "mu", "lv", "z", "hd", "y"):
                assert rel(aux[k], g["s1_" + k]) <= 1e-6, k
            assert rel(aux["logp_rows"], g["s1_logp_rows"]) <= 1e-12
            assert abs(aux["sgvb"] - g["s1_sgvb"]) <= 1e-10 * abs(g["s1_sgvb"])
            assert rel(O.flatten(aux["data_grads"]), g["s1_data_grads"]) <= 1e-6
            assert rel(O.flatten(p), g["theta1"]) <= 1e-6 and rel(O.flatten(a), g["acc1"]) <= 1e-6
    assert rel(O.flatten(p), g["theta10"]) <= 1e-6 and rel(O.flatten(a), g["acc10"]) <= 1e-6
