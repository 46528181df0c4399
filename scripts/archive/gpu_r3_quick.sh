# Round 3 quick loop: the fp32 step's parity tests, then the plain and driver-form MNIST lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_dropin.py tests/test_gpu_golden.py tests/test_gpu_api.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
tail -2 gpurun_out/quick_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/quick_tests.log | head -30; exit 1; }
for i in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/bench_plain$i.json 2> gpurun_out/bench_plain.err || { tail -20 gpurun_out/bench_plain.err; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline --config frey > gpurun_out/bench_frey$i.json 2> gpurun_out/bench_frey.err || { tail -20 gpurun_out/bench_frey.err; exit 1; }
done
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
python3 -c "
import json
for f in ('bench_plain1','bench_plain2','bench_frey1','bench_frey2','bench_driver'):
    d=json.load(open('gpurun_out/%s.json'%f)); print(f, round(d['ms_per_step']*1000,2), 'us/step', {k: round(v*1000,2) for k,v in d['kernels_ms'].items()})"
