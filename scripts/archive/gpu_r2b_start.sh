# Round-2 re-entry: the whole GPU suite, smoke, driver + default bench lines, then the
# config-5 GEMMs against hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_r2_check.sh || exit 1
timeout -k 10 180 python3 scripts/gemm_vs_blas.py > gpurun_out/gemm_vs_blas.txt 2>&1; rc=$?
cat gpurun_out/gemm_vs_blas.txt | tail -8
exit $rc
