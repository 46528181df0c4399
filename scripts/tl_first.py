"""Diagnostics: stage stamps of the MNIST step's FIRST launch (encoder + the previous step's
deferred dW2 workers, latent.hpp enc_latent16_w2_kernel), timeline build (VAEB_TIMELINE):
per slot, min / median / max over the workgroups that wrote it, in 10-ns ticks from the
launch's first stamp.  Encoder workgroups stamp at logical ids [0, 256), the dW2 tile workers
at 256 + tile (wgrad_body slots: 4 batch pointer, 5 panels landed, 2 / 6 staged, 1 MFMA +
K reduction done, 3 epilogue stores issued)."""
import os
import sys

os.environ.setdefault("VAEB_LIB_VARIANT", "tl")
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeb_amd import _lib  # noqa: E402
from vaeb_amd.model import initial_params  # noqa: E402
from vaeb_amd.synthetic import mnist_like  # noqa: E402

D, H, Z, B = 784, 500, 20, 100
ctx = _lib.Context(D, H, Z, B, max_eval_rows=1000, use_graph=False)
ctx.set_data(mnist_like(n=2000, D=D))
ctx.set_params(np.concatenate([a.ravel() for a in initial_params(D, H, Z, False)]))
for i in range(20):
    ctx.update(i % 20)
for rep in range(4):
    tl = ctx.debug_timeline(rep).astype(np.int64)
    print(f"rep {rep}: {tl.shape[0]} launches")
    for k in range(tl.shape[0]):
        s = tl[k]
        used = np.where((s > 0).any(axis=1))[0]
        if not len(used):
            continue
        t0 = s[used][s[used] > 0].min()
        end = s[used].max() - t0
        print(f" launch {k}: wgs={len(used)} end={end}")
        parts = [(0, 256), (256, 1 << 30)] if k == 0 else [(0, 1 << 30)]
        for lo, hi in parts:
            sel = used[(used >= lo) & (used < hi)]
            if not len(sel):
                continue
            print(f"  part [{lo}, {hi}): {len(sel)} wgs")
            for j in range(8):
                v = s[sel, j]
                v = v[v > 0] - t0
                if len(v):
                    print(f"    slot {j}: n={len(v):4d} min={v.min():5d} med={int(np.median(v)):5d} max={v.max():5d}")
