"""Race screen (guide §5: a sync-structure edit makes a new template -- screen it over many
runs at several sizes): the 8-phase 256 x 256 GEMM (test hook, ksplit < 0) against float64
products of the bf16-rounded operands, many runs over shapes, layouts and split-K; counts
the runs whose result misses the bound anywhere."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from oracle import vaeb_oracle as O  # noqa: E402
from vaeb_amd import _lib  # noqa: E402

ctx = _lib.Context(64, 32, 8, 16, dtype=_lib.DTYPE_BF16)
shapes = [(512, 512, 1024, 1), (768, 512, 576, 1), (256, 1024, 2048, 2), (1024, 256, 520, 1), (512, 768, 4096, 4)]
rng = np.random.default_rng(0)
bad = runs = 0
t0 = time.time()
cache = {}
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 120):
    M, N, K, ks = shapes[it % len(shapes)]
    ako, bko = (it // len(shapes)) % 2, (it // (2 * len(shapes))) % 2
    key = (M, N, K)
    if key not in cache:
        A = rng.standard_normal((M, K)).astype(np.float32)
        B = rng.standard_normal((K, N)).astype(np.float32)
        Aq, Bq = O.bf16_round(A).astype(np.float64), O.bf16_round(B).astype(np.float64)
        cache[key] = (A, B, Aq @ Bq, 1e-5 * (np.abs(Aq) @ np.abs(Bq)) + 1e-30)
    A, B, ref, bound = cache[key]
    C = ctx.test_gemm_bf16(A.T.copy() if ako else A, B if bko else B.T.copy(), ako, bko, M, N, K, -ks)
    runs += 1
    miss = int(np.sum(np.abs(C - ref) > bound))
    if miss:
        bad += 1
        print(f"run {it}: {M}x{N}x{K} ks={ks} ako={ako} bko={bko}: {miss} elements off", flush=True)
print(f"gemm8 screen: {bad} of {runs} runs wrong ({time.time() - t0:.0f} s)", flush=True)
sys.exit(1 if bad else 0)
