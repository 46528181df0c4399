"""Diagnostics: the last launch's stage stamps from a timeline dump (gpurun_out/tl_mnist.npz,
scripts/tl_dump.py): the dW3 tiles [0, 416) and the latent reducers (logical ids after the tiles
and the ELBO workgroup), medians in 10-ns ticks from the launch's first workgroup, per rep."""
import sys

import numpy as np

tl = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tl_mnist.npz")["tl"].astype(np.int64)
TILE = {0: "start", 4: "batch ptr", 5: "X landed", 7: "poll returned", 2: "dA3 formed", 6: "LDS staged",
        1: "K loop", 3: "epilogue"}
RED = {0: "start", 5: "slabs landed", 2: "dMu|dLv formed", 6: "stores drained", 3: "end"}
for rep in range(tl.shape[0]):
    s = tl[rep, -1]
    used = np.where(s[:, 0] > 0)[0]
    t0 = s[used, 0].min()

    def med(sel, j):
        v = s[sel, j][s[sel, j] > 0] - t0
        return int(np.median(v)) if len(v) else -1
    tiles = used[used < 416]
    reds = used[used >= 449]
    print(rep, "tiles:", ", ".join(f"{n} {med(tiles, j)}" for j, n in TILE.items()))
    print(rep, "reducers:", ", ".join(f"{n} {med(reds, j)}" for j, n in RED.items()), f"(n={len(reds)})")
