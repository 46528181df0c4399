# Round 4 iteration: the fp32 step parity tests, then a default-vs-switch bench A/B and stage stamps.
# usage: [TL_ENV='ENV=VAL ...'] gpu_r4_iter.sh [ENV=VAL ...]  (the A/B arms besides the default;
# TL_ENV: the environment of the stage-stamp run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_step.py tests/test_gpu_golden.py tests/test_gpu_dropin.py tests/test_gpu_api.py \
  "tests/test_gpu_bf16.py::test_bf16_dp_path_world1_matches_fused_optimizer" > gpurun_out/r4_iter_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_iter_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r4_iter_tests.log | head -20; exit 1; }
AB_ROUNDS=${AB_ROUNDS:-2} bash scripts/env_ab2.sh "$@" || exit 1
if [ -f vaeb_amd/libvaeb_hip_tl.so ]; then
  env $TL_ENV timeout -k 10 120 python3 scripts/tl_dump.py mnist > /dev/null && env $TL_ENV timeout -k 10 120 python3 scripts/tl_stages.py > gpurun_out/tl_stages.txt 2>&1 || exit 1
fi
