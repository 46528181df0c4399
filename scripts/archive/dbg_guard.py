"""Diagnostics: a backward-only overflow of the fixed-point hand-off (Frey 560-200-2) after
the forward-overflow sequence of test_fixed_point_handoff_overflow_is_reported_not_silent."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import vaeb_oracle as O
from vaeb_amd import _lib
cfg = O.Config(D=560, H=200, Z=2, continuous=True)
x = O.synthetic_frey(n=300)
theta0 = O.flatten(O.init_params(cfg))
sl = O.unflatten(np.arange(theta0.size), cfg)


def step(ctx, tag, fn):
    try:
        v = fn(); print(tag, "ok", v, flush=True)
    except _lib.VaebError as e:
        print(tag, "ERR", str(e)[:70], flush=True)


for history in (False, True):
    ctx = _lib.Context(560, 200, 2, 100, decoder=_lib.DEC_GAUSSIAN, max_eval_rows=100)
    ctx.set_data(x); ctx.set_params(theta0); ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
    step(ctx, "good", lambda: ctx.update(0))
    if history:
        bad = theta0.copy(); bad[sl[0].ravel()] = 1.0; bad[sl[1].ravel()] = np.nan
        ctx.set_params(bad)
        step(ctx, "w4nan", lambda: ctx.update(1))
        ctx.set_params(bad); ctx.update_many(np.array([1, 2], np.int32))
        step(ctx, "w4nan_many", lambda: ctx.epoch_elbo())
        ctx.set_params(theta0); ctx.set_adagrad_state(np.zeros_like(theta0))
        step(ctx, "good2", lambda: ctx.update(0))
        step(ctx, "elbo", lambda: ctx.epoch_elbo())
    for name, idx, val in (("w6_nan", 5, np.nan), ("w6_huge", 5, 1e4), ("w2_huge", 4, 1e5)):
        bad = theta0.copy(); bad[sl[idx].ravel()] = val
        ctx.set_params(bad)
        step(ctx, name, lambda: ctx.update(1))
        dml = ctx.activation("dMuLv", 100 * 4)
        print("   dMuLv nan", int(np.isnan(dml).sum()), "mu finite", bool(np.isfinite(ctx.activation("mu", 200)).all()))
        ctx.set_params(theta0); ctx.set_adagrad_state(np.zeros_like(theta0))
        step(ctx, "restore", lambda: ctx.update(0))
    ctx.close()
