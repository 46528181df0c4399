# Round 3: GPU parity suite, then the driver-form, default and --sync bench lines and the call anatomy.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/bench_plain.json 2> gpurun_out/bench_plain.err || { tail -20 gpurun_out/bench_plain.err; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline --sync --steps 2000 --warmup 100 > gpurun_out/bench_sync.json 2> gpurun_out/bench_sync.err || { tail -20 gpurun_out/bench_sync.err; exit 1; }
timeout -k 10 300 python3 scripts/call_anatomy.py > gpurun_out/call_anatomy.txt 2>&1 || { tail -20 gpurun_out/call_anatomy.txt; exit 1; }
cat gpurun_out/call_anatomy.txt
python3 -c "
import json
for f in ('bench_driver','bench_plain','bench_sync'):
    d=json.load(open('gpurun_out/%s.json'%f)); print(f, round(d['ms_per_step']*1000,2), 'us/step', round(d['value']), 'img/s', d.get('graph'))"
