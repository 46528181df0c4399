# Round-2 check: the whole GPU suite (no -x: every failure listed), smoke, the driver's
# bench command and the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest.log
tail -4 gpurun_out/pytest.log
grep -E "FAILED|ERROR" gpurun_out/pytest.log | head -30
# a fault / timeout ends the call here; test failures do not
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
cat gpurun_out/smoke.log
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python3 -c "
import json
for f in ('bench_driver', 'bench_default'):
    d=json.load(open('gpurun_out/%s.json' % f))
    print(f, 'us/step', round(d['ms_per_step']*1000,2), 'img/s', round(d['value']), 'n_gpus', d['n_gpus'])
    print({k: round(v*1000,2) for k,v in d['kernels_ms'].items()})
    print(d.get('cpu_baseline'))"
