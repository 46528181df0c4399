"""Diagnostics: the fixed cost of one synchronised update_many(n) call (MNIST 784-500-20,
B = 100), as the driver's bench times it: for n in a sweep, the host time until
update_many returns (enqueue) and until the stream sync returns (total), median of 15
calls each; a least-squares line total = fixed + n * per_step separates the call's fixed
cost from the step time."""
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
ns = [1, 2, 5, 10, 20, 32, 40, 64]
res = {}
for rep in range(15):
    for n in ns:
        o = rng.integers(0, 500, n).astype(np.int32)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.update_many(o)
        t1 = time.perf_counter()
        ctx.synchronize()
        t2 = time.perf_counter()
        res.setdefault(n, []).append((1e6 * (t1 - t0), 1e6 * (t2 - t0)))
xs, ys = [], []
for n in ns:
    a = np.array(res[n])
    enq, tot = np.median(a[:, 0]), np.median(a[:, 1])
    xs.append(n)
    ys.append(tot)
    print(f"n={n:3d}: enqueue {enq:7.1f} us  total {tot:8.1f} us  = {tot / n:6.2f} us/step", flush=True)
A = np.vstack([np.ones(len(xs)), xs]).T
(fixed, per), *_ = np.linalg.lstsq(A, np.array(ys), rcond=None)
print(f"fit: fixed {fixed:.1f} us + {per:.2f} us/step")
