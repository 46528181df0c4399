"""Diagnostics (round 3): the fp32 DP step at world 1 with bucket A forked onto the second
stream (VAEB_DP_OVERLAP=1) for a kernel trace: 64 steps in one call after a warm-up (run under
rocprofv3 --kernel-trace; scripts/trace_gaps.py reads the gaps)."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
os.environ.setdefault("VAEB_DP_OVERLAP", "1")
from vaeb_amd import _lib  # noqa: E402
from vaeb_amd.model import initial_params  # noqa: E402
from vaeb_amd.synthetic import mnist_like  # noqa: E402

ctx = _lib.Context(784, 500, 20, 100, max_eval_rows=100)
if not os.environ.get("VAEB_DP_NOCOMM"):   # (set: the fused step without a communicator, for reference)
    ctx.comm_init(_lib.Context.comm_unique_id(), 0, 1)
ctx.set_data(mnist_like(n=50000))
ctx.set_params(np.concatenate([a.ravel() for a in initial_params(784, 500, 20, False)]))
ctx.set_eps_mode(0, 10)
rng = np.random.default_rng(0)
ctx.update_many(rng.integers(0, 500, 40).astype(np.int32))
ctx.synchronize()
g, _ = ctx.time_update_many(rng.integers(0, 500, 64).astype(np.int32))
print(f"overlap {'none' if os.environ.get('VAEB_DP_NOCOMM') else os.environ['VAEB_DP_OVERLAP']}: "
      f"{g * 1e3 / 64:.2f} us/step", flush=True)
ctx.close()
