# Round check: GPU parity tests, smoke, full bench line, kernel-trace profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest.log
tail -8 gpurun_out/pytest.log
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
cat gpurun_out/smoke.log
timeout -k 10 240 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
cut -c1-1500 gpurun_out/bench_default.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit 1
cut -c1-160 gpurun_out/prof/run_kernel_stats.csv
