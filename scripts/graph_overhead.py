"""Diagnostics: wall time of update_many(n) (one host call, sync before and after) for
several n, MNIST 784-500-20 B=100; shows the fixed per-call cost the driver's short
bench (20 timed steps) sees on top of the per-step graph time."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from vaeb_amd import _lib  # noqa: E402
from vaeb_amd.model import initial_params  # noqa: E402
from vaeb_amd.synthetic import mnist_like  # noqa: E402

ctx = _lib.Context(784, 500, 20, 100, max_eval_rows=100)
ctx.set_data(mnist_like(n=50000))
ctx.set_params(np.concatenate([a.ravel() for a in initial_params(784, 500, 20, False)]))
ctx.set_eps_mode(0, 10)
rng = np.random.default_rng(0)
t0 = time.perf_counter()
ctx.update_many(rng.integers(0, 500, 64).astype(np.int32))   # captures the graph family
ctx.synchronize()
print(f"first call (64 steps, graph capture included): {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
for n in [1, 2, 4, 5, 8, 16, 19, 20, 32, 64, 128, 1000]:
    ts = []
    for rep in range(15):
        o = rng.integers(0, 500, n).astype(np.int32)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.update_many(o)
        ctx.synchronize()
        ts.append(time.perf_counter() - t0)
    t = np.median(ts) * 1e6
    tmin = np.min(ts) * 1e6
    print(f"n={n:5d}  call median {t:9.1f} us (min {tmin:9.1f})  per step {t / n:7.2f} us", flush=True)
