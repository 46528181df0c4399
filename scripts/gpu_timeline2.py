"""Diagnostics: per-launch, per-part (phase tiles vs weight-gradient tiles) end times of
one eager MNIST 784-500-20 step (10 ns ticks from the launch's first workgroup start)."""
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
# phase tiles first in the fused grids: launch 2 = 224 PDhd tiles, launch 3 = 7 row blocks
parts = {2: 224, 3: 7}
for rep in range(2):
    tl = ctx.debug_timeline(rep).astype(np.int64)
    prev_end = None
    for k in range(tl.shape[0]):
        s = tl[k]
        used = np.where(s[:, 0] > 0)[0]
        if not len(used):
            continue
        t0 = s[used, 0].min()
        ends = np.array([max(v for v in s[w, :6] if v > 0) for w in used]) - t0
        gap = (t0 - prev_end) if prev_end is not None else 0
        prev_end = t0 + ends.max()
        line = (f"rep {rep} launch {k}: wgs={len(used)} gap={gap} start-spread={s[used, 0].max() - t0} "
                f"end max={ends.max()} med={int(np.median(ends))}")
        if k in parts:
            n = parts[k]
            ph = used < n
            line += f" | phase end max={ends[ph].max()} med={int(np.median(ends[ph]))}"
            line += f" | wgrad end max={ends[~ph].max()} med={int(np.median(ends[~ph]))}"
            w = used[~ph]
            sl = [f"s{j}:{int(np.median(s[w, j] - s[w, 0]))}" for j in (1, 3) if (s[w, j] > 0).all()]
            line += " wgrad " + " ".join(sl)
        print(line)
