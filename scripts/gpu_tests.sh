# Full GPU parity suite (one pytest process), then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/bench_plain.json 2> gpurun_out/bench_plain.err || { tail -20 gpurun_out/bench_plain.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_plain.json'))
print('us/step', round(d['ms_per_step']*1000,2), 'img/s', round(d['value']))
print({k: round(v*1000,2) for k,v in d['kernels_ms'].items()})"
