"""Diagnostics: MNIST step time of the data-parallel code path at world size 1 (gradients
stored, RCCL all-reduce inside the graph, replicated Adagrad) vs the fused-optimizer path."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import vaeb_oracle as O  # noqa: E402
from vaeb_amd import _lib  # noqa: E402

cfg = O.Config(D=784, H=500, Z=20)
x = O.synthetic_mnist(n=50000)
order = np.random.default_rng(1).permutation(500).astype(np.int32)
for use_comm in (False, True, False, True):
    ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, 100, max_eval_rows=500)
    if use_comm:
        ctx.comm_init(_lib.Context.comm_unique_id(), 0, 1)
    ctx.set_data(x)
    ctx.set_params(O.flatten(O.init_params(cfg)))
    ctx.update_many(order[:100])
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.update_many(np.concatenate([order] * 4))
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / 2000
    prof = ctx.profile_steps(20)
    print(f"comm={use_comm}: {dt * 1e6:.2f} us/step", {k: round(v * 1000, 2) for k, v in prof})
    ctx.close()
