"""The HIP path (fp32 engine, through the C ABI) against the committed golden step
vectors (tests/golden/step_golden.npz): 10 steps with the golden's injected eps and batch
order.  Tolerances are SURVEY 8(d)'s: returned SGVB/B 1e-4 relative per step, step-1 data
gradient 1e-4 relative (norm-wise), theta after one step within 1e-3 lr (all but 1e-3 of
the elements; the first Adagrad step is ~lr sign(g), sensitive where |g| ~ 1e-6), the
10-step displacement theta10 - theta0 1e-3 relative, and the decoder mean at z = mu
(VAEB.py:267-270) within 1e-5 absolute."""
import numpy as np
import pytest

from oracle import vaeb_oracle as O
from tests.test_golden import CASES, load, rel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(CASES))
def test_hip_step_matches_golden(name):
    from vaeb_amd import _lib
    g = load(name)
    cfg = O.Config(**CASES[name])
    B = int(g["B"])
    ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, L=cfg.L,
                       decoder=_lib.DEC_GAUSSIAN if cfg.continuous else _lib.DEC_BERNOULLI,
                       estimator=_lib.EST_LA if cfg.estimator == "LA" else _lib.EST_LB,
                       objective=_lib.OBJ_MEAN_MAP if cfg.objective == "mean_map" else _lib.OBJ_SUM_PRIOR,
                       keep_grads=True, max_eval_rows=B)
    ctx.set_data(g["x"])
    ctx.set_params(g["theta0"])
    y = ctx.reconstruct(g["x"][:B])
    assert np.abs(y - g["y_mean_b0"]).max() <= 1e-5
    ctx.set_eps_mode(_lib.EPS_HOST)
    for s, b in enumerate(g["order"]):
        ctx.push_eps(g["eps"][s])
        e = ctx.update(int(b))
        assert abs(e - g["elbos"][s]) <= 1e-4 * abs(g["elbos"][s]), (s, e, g["elbos"][s])
        if s == 0:
            assert rel(ctx.get_grads(), g["s1_data_grads"]) <= 1e-4
            d = np.abs(ctx.get_params() - g["theta1"])
            assert d.max() <= 2 * cfg.lr + 1e-7
            assert float((d > 1e-3 * cfg.lr).mean()) <= 1e-3
            assert rel(ctx.get_adagrad_state(), g["acc1"]) <= 1e-3
    assert rel(ctx.get_params() - g["theta0"], g["theta10"].astype(np.float64) - g["theta0"]) <= 1e-3
    ctx.close()


@pytest.mark.parametrize("name", ["mnist_lb", "mnist_mean_map"])
def test_bf16_engine_tracks_golden(name):
    """The bf16 engine (bf16 operands, fp32 accumulation and master weights) on the same
    10 steps: SGVB/B within 1e-2 relative for the first 3 steps and the step-1 data
    gradient within 8e-2 (norm-wise) of the float64 golden -- test_gpu_bf16.py's bounds vs
    the unquantised restatement; after that the two Adagrad trajectories have separated
    (~lr sign(g) steps), so steps 4-10 are only held to 5e-2 (mnist_mean_map: 1.0e-2 at
    step 7, 3.2e-2 at step 10)."""
    from vaeb_amd import _lib
    g = load(name)
    cfg = O.Config(**CASES[name])
    B = int(g["B"])
    ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, objective=_lib.OBJ_MEAN_MAP if cfg.objective == "mean_map"
                       else _lib.OBJ_SUM_PRIOR, keep_grads=True, max_eval_rows=B, dtype=_lib.DTYPE_BF16)
    ctx.set_data(g["x"])
    ctx.set_params(g["theta0"])
    ctx.set_eps_mode(_lib.EPS_HOST)
    for s, b in enumerate(g["order"]):
        ctx.push_eps(g["eps"][s])
        e = ctx.update(int(b))
        tol = 1e-2 if s < 3 else 5e-2
        assert abs(e - g["elbos"][s]) <= tol * abs(g["elbos"][s]), (s, e, g["elbos"][s])
        if s == 0:
            assert rel(ctx.get_grads(), g["s1_data_grads"]) <= 8e-2
    ctx.close()
