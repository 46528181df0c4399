"""Diagnostics: a few config-5 (4096-2048-128, B = 8192, bf16) training steps through
update_many and nothing else, for a rocprofv3 kernel trace of the forked step
(scripts/trace_timeline.py prints the last launches with their queues)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeb_amd import _lib  # noqa: E402
from vaeb_amd.model import initial_params  # noqa: E402

D, H, Z, B = 4096, 2048, 128, 8192
n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
rng = np.random.default_rng(0)
x = (rng.random((4 * B, D)) < 0.3).astype(np.float32)
ctx = _lib.Context(D, H, Z, B, max_eval_rows=B, dtype=_lib.DTYPE_BF16)
ctx.set_data(x)
ctx.set_params(np.concatenate([a.ravel() for a in initial_params(D, H, Z, False)]))
ctx.update_many(np.arange(n, dtype=np.int32) % 4)
print("elbo", ctx.epoch_elbo())
ctx.close()
