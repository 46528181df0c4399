"""Diagnostics (round 6): the fixed cost of a short update_many call for the library this process
loads (VAEB_LIB_VARIANT selects an A/B build): MNIST 784-500-20 B=100, a fresh context, warm-up,
then 40 calls of 20 steps each -- median wall time (call + synchronize) and median GPU time
(events on the context's stream around the call); then 5 calls of 1000 steps for the steady rate."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeb_amd import _lib  # noqa: E402
from vaeb_amd.model import initial_params  # noqa: E402
from vaeb_amd.synthetic import mnist_like  # noqa: E402

ctx = _lib.Context(784, 500, 20, 100, max_eval_rows=100)
ctx.set_data(mnist_like(n=50000))
ctx.set_params(np.concatenate([a.ravel() for a in initial_params(784, 500, 20, False)]))
ctx.set_eps_mode(0, 10)
rng = np.random.default_rng(0)
ctx.update_many(rng.integers(0, 500, 64).astype(np.int32))
ctx.synchronize()
ctx.busy(30000)
walls, gpus = [], []
for rep in range(40):
    o = rng.integers(0, 500, 20).astype(np.int32)
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.update_many(o)
    ctx.synchronize()
    walls.append(time.perf_counter() - t0)
    g, _ = ctx.time_update_many(rng.integers(0, 500, 20).astype(np.int32))
    gpus.append(g * 1e-3)
steady = min(ctx.time_update_many(rng.integers(0, 500, 1000).astype(np.int32))[0] for _ in range(5))
print(f"{os.environ.get('VAEB_LIB_VARIANT', 'new'):5s} 20-step call: wall {1e6 * np.median(walls):6.1f} us "
      f"({1e6 * np.median(walls) / 20:.2f}/step), gpu {1e6 * np.median(gpus):6.1f} us "
      f"({1e6 * np.median(gpus) / 20:.2f}/step); 1000-step {steady:.2f} us/step", flush=True)
ctx.close()
