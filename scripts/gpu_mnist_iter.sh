# MNIST fp32 iteration: parity tests, bench line, FETCH_SIZE pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/mn
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mn/tests.log 2>&1; rc=$?
tail -3 gpurun_out/mn/tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/mn/tests.log | head -20; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/mn/bench.json 2> gpurun_out/mn/bench.err || { tail -20 gpurun_out/mn/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/mn/bench.json'))
print('us/step', round(d['ms_per_step']*1000,2), 'img/s', round(d['value']))
print({k: round(v*1000,2) for k,v in d['kernels_ms'].items()})"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/mn/fetch -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > /dev/null 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/mn/fetch.json gpurun_out/mn/fetch | grep vaeb
