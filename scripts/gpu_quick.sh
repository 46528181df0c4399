# Quick GPU iteration: parity tests, plain bench, in-kernel timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py tests/test_gpu_api.py -q -m gpu -x > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest.log
tail -6 gpurun_out/pytest.log
if grep -q -E "illegal memory|core dumped|Aborted|HSA_STATUS|Memory access fault" gpurun_out/pytest.log; then echo "GPU fault: stopping"; exit 1; fi
timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > gpurun_out/bench_plain.json 2> gpurun_out/bench_plain.err || exit 1
cut -c1-200 gpurun_out/bench_plain.json; python3 -c "import json;d=json.load(open('gpurun_out/bench_plain.json'));print(d['kernels_ms'])"
timeout -k 10 120 python3 scripts/gpu_timeline.py > gpurun_out/timeline.txt 2>&1
tail -16 gpurun_out/timeline.txt
