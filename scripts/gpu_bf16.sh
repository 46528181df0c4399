# bf16 engine: GEMM layout tests, then step parity tests (stop at the first failure).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 120 --timeout-method thread -k gemm > gpurun_out/bf16_gemm.log 2>&1; rc=$?
tail -5 gpurun_out/bf16_gemm.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 200 --timeout-method thread -k "not gemm" > gpurun_out/bf16_step.log 2>&1; rc=$?
tail -25 gpurun_out/bf16_step.log
exit $rc
