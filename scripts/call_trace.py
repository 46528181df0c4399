"""Diagnostics: one update_many(20) call (MNIST 784-500-20, B=100) repeated, meant to run
under `rocprofv3 --kernel-trace --runtime-trace`; scripts/call_gaps.py then reads the
kernel timestamps to split the call's fixed cost (order upload, graph-to-graph gaps)."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
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
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for rep in range(8):
    o = rng.integers(0, 500, n).astype(np.int32)
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.update_many(o)
    ctx.synchronize()
    print(f"rep {rep}: {1e6 * (time.perf_counter() - t0):.1f} us", flush=True)
