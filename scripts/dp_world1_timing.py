"""Diagnostics: MNIST step time of the data-parallel code path at world size 1 (gradients
stored, RCCL all-reduce inside the graph, replicated Adagrad) vs the fused-optimizer path."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import vaeb_oracle as O  # noqa: E402
from vaeb_amd import _lib  # noqa: E402

BF16 = "--bf16" in sys.argv   # config 5 shapes on the bf16 engine
if BF16:
    cfg, B = O.Config(D=4096, H=2048, Z=128), 8192
    x = (np.random.default_rng(3).random((4 * B, cfg.D)) < 0.5).astype(np.float32)
    order = np.array([0, 1, 2, 3] * 10, np.int32)
else:
    cfg, B = O.Config(D=784, H=500, Z=20), 100
    x = O.synthetic_mnist(n=50000)
    order = np.random.default_rng(1).permutation(500).astype(np.int32)
for use_comm in (False, "0", "1", False, "0", "1"):   # "0"/"1": VAEB_DP_OVERLAP
    ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, max_eval_rows=B if BF16 else 500,
                       dtype=_lib.DTYPE_BF16 if BF16 else _lib.DTYPE_F32)
    if use_comm:
        os.environ["VAEB_DP_OVERLAP"] = use_comm
        ctx.comm_init(_lib.Context.comm_unique_id(), 0, 1)
    ctx.set_data(x)
    ctx.set_params(O.flatten(O.init_params(cfg)))
    ctx.update_many(order[:8] if BF16 else order[:100])
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.update_many(np.concatenate([order] * 4))
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / (4 * len(order))
    prof = ctx.profile_steps(3 if BF16 else 20)
    print(f"comm={use_comm or '-'} (overlap {use_comm or '-'}): {dt * 1e6:.2f} us/step", {k: round(v * 1000, 2) for k, v in prof})
    ctx.close()
