"""Diagnostics (round 3): A/B of the per-call fixed cost, MNIST 784-500-20 B=100, one process,
interleaved rounds (guide §5.4 rule 24).  Variants are context-creation switches:
VAEB_GRAPH_UPLOAD (hipGraphUpload after instantiation), VAEB_SYNC_EAGER (vaeb_update launches
its step eagerly), VAEB_ELBO_HOST (the step's ELBO written into mapped host memory: vaeb_update
needs no device -> host copy).  Reports per variant: the driver's form (fresh context, warmup
5, then 20 timed steps: wall and GPU time), a steady 20-step call, and update() latency."""
import os
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
VARIANTS = {"base": {}, "upload": {"VAEB_GRAPH_UPLOAD": "1"}, "eager": {"VAEB_SYNC_EAGER": "1"},
            "host": {"VAEB_ELBO_HOST": "1"}, "all": {"VAEB_GRAPH_UPLOAD": "1", "VAEB_SYNC_EAGER": "1", "VAEB_ELBO_HOST": "1"}}
KEYS = ["VAEB_GRAPH_UPLOAD", "VAEB_SYNC_EAGER", "VAEB_ELBO_HOST"]


def fresh(env):
    for k in KEYS:
        os.environ.pop(k, None)
    os.environ.update(env)
    ctx = _lib.Context(784, 500, 20, 100, max_eval_rows=100)
    ctx.set_data(x)
    ctx.set_params(theta)
    ctx.set_eps_mode(0, 10)
    return ctx


res = {k: {"drv_wall": [], "drv_gpu": [], "st_wall": [], "st_gpu": [], "upd": []} for k in VARIANTS}
for rnd in range(4):
    for name, env in VARIANTS.items():
        ctx = fresh(env)
        ctx.update_many(rng.integers(0, 500, 5).astype(np.int32))
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.update_many(rng.integers(0, 500, 20).astype(np.int32))
        ctx.synchronize()
        res[name]["drv_wall"].append(time.perf_counter() - t0)
        g, _ = ctx.time_update_many(rng.integers(0, 500, 20).astype(np.int32))
        res[name]["drv_gpu"].append(g * 1e-3)
        for _ in range(5):
            t0 = time.perf_counter()
            g, _ = ctx.time_update_many(rng.integers(0, 500, 20).astype(np.int32))
            res[name]["st_wall"].append(time.perf_counter() - t0)
            res[name]["st_gpu"].append(g * 1e-3)
        for i in range(100):
            t0 = time.perf_counter()
            ctx.update(int(i % 500))
            res[name]["upd"].append(time.perf_counter() - t0)
        ctx.close()
for name, r in res.items():
    med = {k: np.median(v) * 1e6 for k, v in r.items()}
    print(f"{name:7s}: driver-form 20 steps wall {med['drv_wall']:7.1f} us ({med['drv_wall'] / 20:5.2f}/step), "
          f"next call gpu {med['drv_gpu']:6.1f} | steady 20: wall {med['st_wall']:6.1f} gpu {med['st_gpu']:6.1f} | "
          f"update() median {med['upd']:5.1f} us (min {np.min(r['upd']) * 1e6:5.1f})", flush=True)
