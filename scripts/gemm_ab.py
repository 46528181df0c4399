"""Diagnostics: bf16 GEMM layouts / tile widths at the config-5 shapes, interleaved rounds
in one process (guide §5.4 rule 24).  Prints TFLOP/s per variant (median, min)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeb_amd import _lib  # noqa: E402

ctx = _lib.Context(64, 32, 8, 16, dtype=_lib.DTYPE_BF16)
M = N = 4096
K = 8192
variants = []
for ako in (0, 1):
    for bko in (0, 1):
        for bn in (128, 256):
            variants.append((ako, bko, bn))
shapes = [(8192, 2048, 4096), (2048, 4096, 8192)]
for (M, N, K) in shapes:
    res = {v: [] for v in variants}
    for rnd in range(3):
        for v in variants:
            ms = ctx.bench_gemm_bf16(v[0], v[1], M, N, K, v[2], reps=5)
            res[v].append(2.0 * M * N * K / (ms * 1e-3) / 1e12)
    print(f"M={M} N={N} K={K}")
    for v, r in res.items():
        print(f"  A{'KO' if v[0] else 'KC'} B{'KO' if v[1] else 'KC'} bn={v[2]}: median {np.median(r):7.1f} TF/s  min {min(r):7.1f}", flush=True)
ctx.close()
