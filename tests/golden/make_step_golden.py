"""Writes tests/golden/step_golden.npz: golden vectors of the SGVB step from the float64
restatement (oracle/vaeb_oracle.py), at reduced shapes (SURVEY 8(c) "Golden vectors").

The reference itself cannot run in this container (Theano absent, Python-2 sources;
SURVEY 8(c)), so these vectors are produced by the restatement, whose own pins to the
reference's outputs are tests/test_oracle_pins.py (FV trace, FV .mdl identity, logpdf KAT,
reconstruction JPEGs) and tests/test_oracle_autograd.py (hand-written backward vs autograd).
Committed so that (1) the restatement cannot drift unnoticed (tests/test_golden.py) and
(2) the HIP path is checked against fixed numbers, not only against a live oracle run
(tests/test_gpu_golden.py).

Per case: theta0 = VAEB.initialize_params with RandomState(10) and its duplicated W3 / W4
draws (VAEB.py:50-125), a small dataset, a 10-step batch order, the injected eps of each
step, and in float64: step-1 intermediates (h, mu, lv, z, hd, y, per-row log p and KL / LA
terms, SGVB), the step-1 data gradient, theta / acc after 1 and after 10 steps
(Adagrad, VAEB.py:426-444), the 10 returned values SGVB/B (VAEB.py:408-415), and the
decoder mean at z = mu for the first batch (VAEB.py:267-270).  Arrays are stored as
float32 except the scalars and per-row terms (float64).

    python tests/golden/make_step_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import vaeb_oracle as O  # noqa: E402

CASES = {
    # name: (Config kwargs, B, rows in the dataset)
    "mnist_lb": (dict(D=784, H=32, Z=8), 16, 64),
    "frey_la_l2": (dict(D=560, H=32, Z=2, continuous=True, estimator="LA", L=2), 16, 64),
    "mnist_mean_map": (dict(D=784, H=32, Z=8, objective="mean_map"), 16, 64),
}
STEPS = 10


def make_case(kw, B, n):
    cfg = O.Config(**kw)
    x = O.synthetic_frey(n=n, D=cfg.D) if cfg.continuous else O.synthetic_mnist(n=n, D=cfg.D)
    theta0 = O.init_params(cfg)
    rng = np.random.default_rng(20)
    order = rng.integers(0, n // B, STEPS).astype(np.int32)
    eps = rng.standard_normal((STEPS, cfg.L, B, cfg.Z)).astype(np.float32)
    p = [t.astype(np.float64) for t in theta0]
    a = [np.zeros_like(t) for t in p]
    out = dict(x=x, theta0=O.flatten(theta0), order=order, eps=eps, B=np.int32(B))
    elbos = []
    for s in range(STEPS):
        xb = x[order[s] * B:(order[s] + 1) * B].astype(np.float64)
        e, p, a, aux = O.step(p, a, xb, eps[s].astype(np.float64), cfg)
        elbos.append(e)
        if s == 0:
            for k in ("h", "mu", "lv", "z", "hd", "y"):
                out["s1_" + k] = aux[k].astype(np.float32)
            out["s1_logp_rows"] = aux["logp_rows"]
            out["s1_" + ("la_rows" if cfg.estimator == "LA" else "kl_rows")] = aux[
                "la_rows" if cfg.estimator == "LA" else "kl_rows"]
            out["s1_sgvb"] = np.float64(aux["sgvb"])
            out["s1_data_grads"] = O.flatten(aux["data_grads"]).astype(np.float32)
            out["theta1"] = O.flatten(p).astype(np.float32)
            out["acc1"] = O.flatten(a).astype(np.float32)
    out["elbos"] = np.array(elbos, np.float64)
    out["theta10"] = O.flatten(p).astype(np.float32)
    out["acc10"] = O.flatten(a).astype(np.float32)
    p0 = [t.astype(np.float64) for t in theta0]
    x0 = x[:B].astype(np.float64)
    fwd = O.forward_backward(p0, x0, np.zeros((1, B, cfg.Z)), cfg, need_grad=False)
    out["y_mean_b0"] = fwd["y"].astype(np.float32)
    return out


def main():
    arrays = {}
    for name, (kw, B, n) in CASES.items():
        for k, v in make_case(kw, B, n).items():
            arrays[f"{name}/{k}"] = v
    dst = os.path.join(HERE, "step_golden.npz")
    np.savez_compressed(dst, **arrays)
    print(dst, os.path.getsize(dst), "bytes,", len(arrays), "arrays")


if __name__ == "__main__":
    main()
