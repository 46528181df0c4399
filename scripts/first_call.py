"""Diagnostics: the driver's bench form in a fresh context (MNIST 784-500-20, B=100):
warmup 5 steps, sync, then five 20-step calls, each synchronised -- the first 20-step call
is the first replay of that graph instance.  Run once per VAEB_GRAPH_UPLOAD setting."""
import os
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
ctx.update_many(rng.integers(0, 500, 5).astype(np.int32))
ctx.synchronize()
ctx.epoch_elbo()
out = []
for i in range(5):
    o = rng.integers(0, 500, 20).astype(np.int32)
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.update_many(o)
    ctx.synchronize()
    out.append(1e6 * (time.perf_counter() - t0) / 20)
print(f"upload={os.environ.get('VAEB_GRAPH_UPLOAD', '1')}: us/step per 20-step call", " ".join(f"{v:.2f}" for v in out))
