# Round 4: guard diagnostics, the new GPU tests, then a short bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/dbg_guard.py > gpurun_out/dbg_guard.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_cli_dp.py tests/test_gpu_drivers.py \
  "tests/test_gpu_step.py::test_fixed_point_handoff_overflow_is_reported_not_silent" \
  "tests/test_gpu_step.py::test_update_after_async_steps_returns_its_own_value" \
  "tests/test_gpu_bf16.py::test_bf16_full_size_step_matches_rounded_oracle" > gpurun_out/r4_new.log 2>&1
rc=$?; tail -15 gpurun_out/r4_new.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_driver.json')); print(round(d['ms_per_step']*1000,2), 'us/step', d['kernels_ms'])"
