"""Diagnostics: wall time of one update_many(20) call (MNIST 784-500-20, B=100) after the
GPU idled 0.5 s, preceded by (a) a 5-step call, as in the driver's --warmup 5, or (b) a
2000-step call (~90 ms of work) -- separates the call's fixed cost from clock ramp-up."""
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
ctx.update_many(rng.integers(0, 500, 64).astype(np.int32))
ctx.synchronize()


def timed(n):
    o = rng.integers(0, 500, n).astype(np.int32)
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.update_many(o)
    ctx.synchronize()
    return 1e6 * (time.perf_counter() - t0)


for trial in range(4):
    for pre in (5, 2000, 0):
        time.sleep(0.5)
        if pre:
            timed(pre)
        t = timed(20)
        print(f"trial {trial} pre {pre:5d}: 20 steps {t:7.1f} us = {t / 20:5.2f} us/step", flush=True)
