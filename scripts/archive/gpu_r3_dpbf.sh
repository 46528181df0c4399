# Round 3: bf16 DP with the fork -- parity at world 1, then the world-1 DP timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_api.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/dpbf_tests.log 2>&1; rc=$?
tail -2 gpurun_out/dpbf_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/dpbf_tests.log | head -30; exit 1; }
timeout -k 10 400 python3 scripts/dp_world1_timing.py --bf16 > gpurun_out/dp_world1_bf16.txt 2>&1 || { tail -20 gpurun_out/dp_world1_bf16.txt; exit 1; }
grep "us/step" gpurun_out/dp_world1_bf16.txt | cut -c1-120
