"""Diagnostics: the config-5 GEMMs (4096-2048-128, B = 8192) on this library's 16-bit engine
(bare GEMM, no epilogue) against torch.matmul (hipBLASLt) on the same shapes and operand
layouts.  Interleaved rounds in one process; prints TFLOP/s (median of 3 rounds).
Usage: gemm_vs_blas.py [bf16|fp16]  (the operand type of both sides; default bf16)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeb_amd import _lib  # noqa: E402

# (name, M, N, K, A K-outer?, B K-outer?)
DT = sys.argv[1] if len(sys.argv) > 1 else "bf16"
TORCH_DT = {"bf16": torch.bfloat16, "fp16": torch.float16}[DT]
SHAPES = [("enc X.W3", 8192, 2048, 4096, 0, 1),
          ("dec hd.W2", 8192, 4096, 2048, 0, 1),
          ("dhd dA2.W2^T", 8192, 2048, 4096, 0, 0),
          ("dW2 hd^T.dA2", 2048, 4096, 8192, 1, 1),
          ("dW3 X^T.dA3", 4096, 2048, 8192, 1, 1)]


def blas_ms(M, N, K, ako, bko, reps=10):
    a = torch.randn((K, M) if ako else (M, K), device="cuda", dtype=TORCH_DT)
    b = torch.randn((K, N) if bko else (N, K), device="cuda", dtype=TORCH_DT)
    A = a.t() if ako else a
    B = b if bko else b.t()
    for _ in range(3):
        A @ B
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        A @ B
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


ctx = _lib.Context(64, 32, 8, 16, dtype=_lib.DTYPE_F16 if DT == "fp16" else _lib.DTYPE_BF16)
print("operands:", DT)
for name, M, N, K, ako, bko in SHAPES:
    fl = 2.0 * M * N * K
    modes = (128, 256, 8, 9) if ako and bko else (128, 256, 8)   # 9: 8-phase, two K slices combined
    ours = {bn: [] for bn in modes}
    blas = []
    for rnd in range(3):
        for bn in modes:
            ours[bn].append(fl / (ctx.bench_gemm_bf16(ako, bko, M, N, K, bn, reps=10) * 1e-3) / 1e12)
        blas.append(fl / (blas_ms(M, N, K, ako, bko) * 1e-3) / 1e12)
    print(f"{name:14s} M={M} N={N} K={K}: ours bn128 {np.median(ours[128]):6.0f}  bn256 {np.median(ours[256]):6.0f}"
          f"  8-phase 256 {np.median(ours[8]):6.0f}"
          + (f"  8-phase 2-slice {np.median(ours[9]):6.0f}" if 9 in ours else "") +
          f"  hipBLASLt {np.median(blas):6.0f} TF/s", flush=True)
ctx.close()
