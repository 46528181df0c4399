# bf16 iteration: parity tests, then the config-5 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/synth
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1; rc=$?
tail -4 gpurun_out/bf16_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/bf16_tests.log | head -20; exit 1; }
timeout -k 10 300 python3 bench.py --config synth --no-cpu-baseline > gpurun_out/synth/bench_iter.json 2> gpurun_out/synth/bench_iter.err || { tail -20 gpurun_out/synth/bench_iter.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/synth/bench_iter.json'))
print('ms/step', round(d['ms_per_step'],4), 'img/s', round(d['value']), 'TF/s', round(d['step_tflops'],1))
print({k: round(v*1000,1) for k,v in d['kernels_ms'].items()})"
