"""Diagnostics: per-launch stage stamps of one eager MNIST 784-500-20 step (10 ns ticks
from the launch's first workgroup start): for every stamp slot, min / median / max over
the workgroups that wrote it."""
import os
import sys

# the stamps exist only in the VAEB_TIMELINE build (__graft_entry__.build_variant('tl', 'VAEB_TIMELINE'))
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
# stamp ranges per launch: the folded step (4 launches) stamps the dhd tiles at logical ids
# [0, 224) and the dW2 tiles after them; its last launch: dW3 [0, 416), dW45, dW1, ELBO
PARTS = {(False, 2): [(0, 224), (224, 1 << 30)], (False, 3): [(0, 416), (416, 440), (440, 448), (448, 1 << 30)],
         (True, 2): [(0, 224), (224, 1 << 30)]}
for rep in range(3):
    tl = ctx.debug_timeline(rep).astype(np.int64)
    prev = None
    for k in range(tl.shape[0]):
        s = tl[k]
        used = np.where(s[:, 0] > 0)[0]
        if not len(used):
            continue
        t0 = s[used, 0].min()
        end = max(s[w][s[w] > 0].max() for w in used) - t0
        print(f"rep {rep} launch {k}: wgs={len(used)} gap={(t0 - prev) if prev is not None else 0} end={end}")
        prev = t0 + end
        parts = PARTS.get((tl.shape[0] > 4, k), [(0, 1 << 30)])
        for lo, hi in parts:
            sel = used[(used >= lo) & (used < hi)]
            if not len(sel):
                continue
            print(f"  part [{lo}, {hi}): {len(sel)} wgs")
            for j in range(8):
                v = s[sel, j]
                v = v[v > 0] - t0
                if len(v) and j != 7:
                    print(f"    slot {j}: n={len(v):4d} min={v.min():5d} med={int(np.median(v)):5d} max={v.max():5d}")
