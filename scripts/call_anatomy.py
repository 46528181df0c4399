"""Diagnostics (round 3): where a short update_many call's time goes, MNIST 784-500-20 B=100.
For n steps: wall time of the call + sync, the host's enqueue time, and the GPU time between
events bracketing the call on the context's stream.  Run in the driver's form too: a fresh
context, 5 warmup steps, then 20 timed."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from vaeb_amd import _lib  # noqa: E402
from vaeb_amd.model import initial_params  # noqa: E402
from vaeb_amd.synthetic import mnist_like  # noqa: E402

x = mnist_like(n=50000)
theta = np.concatenate([a.ravel() for a in initial_params(784, 500, 20, False)])
rng = np.random.default_rng(0)


def fresh():
    ctx = _lib.Context(784, 500, 20, 100, max_eval_rows=100)
    ctx.set_data(x)
    ctx.set_params(theta)
    ctx.set_eps_mode(0, 10)
    return ctx


# driver form: fresh context, warmup 5 (captures), then 20; "busy" variants first keep
# every CU busy for that many ms (is the extra the clock ramp after the host-bound capture?)
for trial in range(6):
    busy_ms = [0, 5, 30][trial % 3]
    ctx = fresh()
    if busy_ms:
        ctx.update_many(rng.integers(0, 500, 1).astype(np.int32))   # capture first (host-bound, GPU idle)
        ctx.synchronize()
        ctx.busy(busy_ms * 1000)
    t0 = time.perf_counter()
    ctx.update_many(rng.integers(0, 500, 5).astype(np.int32))
    ctx.synchronize()
    tw = time.perf_counter() - t0
    o = rng.integers(0, 500, 20).astype(np.int32)
    t0 = time.perf_counter()
    g, h = ctx.time_update_many(o)
    t = time.perf_counter() - t0
    g2, h2 = ctx.time_update_many(rng.integers(0, 500, 20).astype(np.int32))
    g3, h3 = ctx.time_update_many(rng.integers(0, 500, 1000).astype(np.int32))
    print(f"driver form {trial} (busy {busy_ms} ms): warmup call {tw * 1e3:.1f} ms; 20 steps wall {t * 1e6:.0f} us, gpu {g * 1e3:.0f} us, "
          f"enqueue {h * 1e3:.0f} us | again gpu {g2 * 1e3:.0f} us (enq {h2 * 1e3:.0f}) | 1000: {g3:.2f} ms "
          f"= {g3:.4f} us/step x1000 (enq {h3:.2f} ms)", flush=True)
    ctx.close()
ctx = fresh()
ctx.update_many(rng.integers(0, 500, 64).astype(np.int32))
ctx.synchronize()
for n in (1, 5, 20, 32, 33, 100, 1000):
    gs, hs, ws = [], [], []
    for rep in range(10):
        o = rng.integers(0, 500, n).astype(np.int32)
        t0 = time.perf_counter()
        g, h = ctx.time_update_many(o)
        ws.append(time.perf_counter() - t0)
        gs.append(g)
        hs.append(h)
    print(f"n={n:5d}: wall {np.median(ws) * 1e6:8.1f} us  gpu {np.median(gs) * 1e3:8.1f} us ({np.median(gs) * 1e3 / n:6.2f}/step)"
          f"  enqueue {np.median(hs) * 1e3:7.1f} us", flush=True)
# synchronous update() as the reference calls it
ts = []
for i in range(200):
    t0 = time.perf_counter()
    ctx.update(int(i % 500))
    ts.append(time.perf_counter() - t0)
print(f"update(): median {np.median(ts) * 1e6:.1f} us, min {np.min(ts) * 1e6:.1f} us", flush=True)
