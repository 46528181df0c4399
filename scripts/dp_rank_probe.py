"""Diagnostics: where a sharded-DP rank's bf16 shadow differs from bf16(theta') (vaeb_dp_rank_update)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import vaeb_oracle as O
from vaeb_amd import _lib

D, H, Z = 512, 264, 40
ctx = _lib.Context(D, H, Z, 64, max_eval_rows=64, dtype=_lib.DTYPE_BF16)
P = ctx.P
n_w = P - (H + 2 * Z + H + D)
rng = np.random.default_rng(1)
theta0 = (0.01 * rng.standard_normal(P)).astype(np.float32)
acc0 = (0.1 * np.abs(rng.standard_normal(P))).astype(np.float32)
gsum = rng.standard_normal(P + 1).astype(np.float32)
bits = lambda x: (O.bf16_round(np.asarray(x, np.float32)).view(np.uint32) >> 16).astype(np.uint16)


def run(world, rank, buckets, thg):
    ctx.set_params(theta0)
    ctx.set_adagrad_state(acc0)
    for i, b in enumerate(buckets):
        ctx.dp_rank_update(world, rank, b, gsum, thg, finish=(i == len(buckets) - 1))
    return ctx.get_params(), ctx.get_shadow(n_w)


th_rep, sh_rep = run(1, 0, [2], None)
print("replicated shadow ok:", np.array_equal(sh_rep, bits(th_rep[:n_w])))
for buckets in ([2], [0, 1], [0], [1]):
    for world in (2, 3):
        for rank in range(world):
            th, sh = run(world, rank, buckets, th_rep)
            want = bits(th[:n_w])
            bad = np.flatnonzero(sh != want)
            nanw = int((sh[bad] == 0xFFFF).sum())
            zw = int((sh[bad] == 0).sum())
            runs = []
            if bad.size:
                br = np.flatnonzero(np.diff(bad) != 1)
                starts = np.r_[bad[0], bad[br + 1]]
                ends = np.r_[bad[br], bad[-1]]
                runs = list(zip(starts[:6].tolist(), ends[:6].tolist()))
            print(f"buckets {buckets} world {world} rank {rank}: {bad.size} bad ({nanw} still NaN, {zw} zero) runs {runs} n_runs {len(starts) if bad.size else 0}")
            plan = [_lib.dp_plan(D, H, Z, world, rank, bucket=b) for b in buckets]
            if bad.size:
                print("   plan own", [p["own"] for p in plan], "foreign", [p["foreign"] for p in plan])
