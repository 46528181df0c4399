"""Diagnostics: per-launch in-kernel timeline of one eager SGVB step (MNIST 784-500-20)."""
import os
import sys

# the stamps exist only in the VAEB_TIMELINE build (__graft_entry__.build_variant('tl', 'VAEB_TIMELINE'))
os.environ.setdefault("VAEB_LIB_VARIANT", "tl")

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import vaeb_oracle as O  # noqa: E402
from vaeb_amd import _lib  # noqa: E402

D, H, Z, B = 784, 500, 20, 100
x = O.synthetic_mnist(n=2000, D=D)
ctx = _lib.Context(D, H, Z, B, max_eval_rows=1000, use_graph=False)
ctx.set_data(x)
ctx.set_params(O.flatten(O.init_params(O.Config(D=D, H=H, Z=Z))))
for i in range(20):
    ctx.update(i % 20)
for rep in range(3):
    tl = ctx.debug_timeline(rep).astype(np.int64)
    # s_memtime (shader clock) stamps live in slots 6/7 of tile_body launches; realtime
    # stamps (100 MHz) everywhere else -- keep t0 on the realtime ones
    rt = tl[:, :, :6]
    t0 = rt[rt > 0].min()
    print(f"--- rep {rep} (units: 10 ns ticks from first stamp)")
    for k in range(tl.shape[0]):
        s = tl[k]
        used = s[:, 0] > 0
        if not used.any():
            continue
        s = s[used]
        memtime = (s[:, 6] > 0).any() and np.median(s[:, 6]) < t0 / 2
        cols = []
        for slot in range(8):
            v = s[:, slot]
            v = v[v > 0]
            if len(v) and not (memtime and slot >= 6):
                cols.append(f"s{slot}[{(v.min()-t0):5d}..{(v.max()-t0):5d}]")
        print(f"launch {k}: wgs={used.sum():4d} " + " ".join(cols))
        rel = []
        for slot in range(1, 8):
            if memtime and slot >= 6:
                continue
            ok = (s[:, slot] > 0)
            if ok.sum() > 0:
                rel.append(f"s{slot}:{np.median(s[ok, slot] - s[ok, 0]):.0f}")
        print("          median ticks since s0:", " ".join(rel))
        if memtime and (s[:, 7] > 0).all() and (s[:, 3] > 0).all():
            clk = np.median((s[:, 7] - s[:, 6]) / np.maximum(s[:, 3] - s[:, 0], 1)) * 100
            print(f"          shader clock ~ {clk:.0f} MHz")
