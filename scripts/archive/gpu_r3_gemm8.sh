# Round 3: the 8-phase bf16 GEMM -- layouts / tails / split-K tests, a race screen, the step
# agreement test, then TFLOP/s against the BK = 32 ring and hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm8 or gemm_layouts" > gpurun_out/gemm8_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gemm8_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gemm8_tests.log | head -30; exit 1; }
timeout -k 10 300 python3 scripts/gemm8_screen.py 150 > gpurun_out/gemm8_screen.txt 2>&1; rc=$?
tail -5 gpurun_out/gemm8_screen.txt
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python3 scripts/gemm_vs_blas.py > gpurun_out/gemm_vs_blas.txt 2>&1 || { tail -20 gpurun_out/gemm_vs_blas.txt; exit 1; }
cat gpurun_out/gemm_vs_blas.txt
