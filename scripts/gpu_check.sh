set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_step.py -x -q -m gpu > gpurun_out/r1_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r1_pytest.log
tail -5 gpurun_out/r1_pytest.log
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --cpu-budget 5 > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.err && cat gpurun_out/r1_bench.json
