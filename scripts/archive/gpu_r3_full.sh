# Round-3 full check: the whole GPU suite, then the evidence of every bench config
# (scripts/gpu_evidence.sh) and the driver-form bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash scripts/gpu_evidence.sh > gpurun_out/evidence.log 2>&1 || { tail -30 gpurun_out/evidence.log; exit 1; }
grep -E "^(mnist|frey|fv|fvs|synth) " gpurun_out/evidence.log
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/round/profiles/driver_form_bench_line.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/round/profiles/driver_form_bench_line.json')); print('driver form', round(d['ms_per_step']*1000,2), 'us/step', d['roofline']['kernel'], round(d['roofline']['frac'],4))"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --sync --steps 2000 --warmup 100 > gpurun_out/round/profiles/sync_bench_line.json 2> gpurun_out/bench_sync.err || { tail -20 gpurun_out/bench_sync.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2000 --warmup 200 > gpurun_out/round/profiles/mnist_plain_bench_line.json 2> gpurun_out/bench_plain.err || { tail -20 gpurun_out/bench_plain.err; exit 1; }
timeout -k 10 300 python3 scripts/dp_world1_timing.py > gpurun_out/round/profiles/dp_world1.txt 2>&1 || { tail -20 gpurun_out/round/profiles/dp_world1.txt; exit 1; }
python3 -c "
import json
for f in ('sync_bench_line', 'mnist_plain_bench_line'):
    d=json.load(open('gpurun_out/round/profiles/%s.json' % f)); print(f, round(d['ms_per_step']*1000,2), 'us/step')"
grep "comm=" gpurun_out/round/profiles/dp_world1.txt
