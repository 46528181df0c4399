"""Diagnostics: the config-5 encoder and dhd GEMM shapes, this engine's 8-phase 256^2 kernel
(bare, fp16 operands) and torch.matmul (hipBLASLt) on the same shapes, 5 launches each, for
rocprofv3 --pmc passes that compare the two kernels counter by counter
(scripts/gpu_gemm_pmc.sh).  Usage: gemm_pmc_probe.py [fp16|bf16]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeb_amd import _lib  # noqa: E402

DT = sys.argv[1] if len(sys.argv) > 1 else "fp16"
TORCH_DT = {"bf16": torch.bfloat16, "fp16": torch.float16}[DT]
SHAPES = [("enc", 8192, 2048, 4096, 0, 1), ("dhd", 8192, 2048, 4096, 0, 0)]
ctx = _lib.Context(64, 32, 8, 16, dtype=_lib.DTYPE_F16 if DT == "fp16" else _lib.DTYPE_BF16)
for name, M, N, K, ako, bko in SHAPES:
    ms = ctx.bench_gemm_bf16(ako, bko, M, N, K, 8, reps=5)
    a = torch.randn((K, M) if ako else (M, K), device="cuda", dtype=TORCH_DT)
    b = torch.randn((K, N) if bko else (N, K), device="cuda", dtype=TORCH_DT)
    A = a.t() if ako else a
    B = b if bko else b.t()
    for _ in range(5):
        A @ B
    torch.cuda.synchronize()
    print(name, "ours", round(2.0 * M * N * K / ms / 1e9), "TF/s", flush=True)
ctx.close()
