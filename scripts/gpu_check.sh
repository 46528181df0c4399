# GPU check: parity tests, plain bench, kernel-trace profile of a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_step.py -q -m gpu > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest.log
tail -15 gpurun_out/pytest.log
if grep -q -E "illegal memory|core dumped|Aborted|HSA_STATUS" gpurun_out/pytest.log; then echo "GPU fault: stopping"; exit 1; fi
timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > gpurun_out/bench_plain.json 2> gpurun_out/bench_plain.err || exit 1
cat gpurun_out/bench_plain.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
echo "rocprof rc=$?"
cat gpurun_out/prof/run_kernel_stats.csv | cut -c1-160
