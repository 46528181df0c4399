"""Diagnostics: MNIST steps with the recomputed latent backward (VAEB_BWD_FX=1) against the
reducer form (=0) from the same state, per step form (update / update_many, dW2 deferred or
not): the ELBO and the parameters after 3 steps."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import vaeb_oracle as O  # noqa: E402
from vaeb_amd import _lib  # noqa: E402

cfg = O.Config(D=784, H=500, Z=20)
x = O.synthetic_mnist(n=800)
for many in (False, True):
    for defer in ("0", "1"):
        for graph in ((False, True) if many else (False,)):
            out = {}
            for fx in ("0", "1"):
                os.environ["VAEB_BWD_FX"] = fx
                os.environ["VAEB_DW2_DEFER"] = defer
                ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, 100, max_eval_rows=100, use_graph=graph)
                ctx.set_data(x)
                ctx.set_params(O.flatten(O.init_params(cfg)))
                ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
                ctx.set_step(0)
                if many:
                    ctx.update_many(np.array([0, 1, 2], np.int32))
                    e = ctx.epoch_elbo()[0]
                else:
                    e = sum(ctx.update(i) for i in range(3))
                out[fx] = (e, ctx.get_params())
                ctx.close()
            d = np.abs(out["0"][1] - out["1"][1]).max()
            print(f"many={many} defer={defer} graph={graph}: elbo {out['0'][0]:.4f} {out['1'][0]:.4f}  max dtheta {d:.3g}", flush=True)
