# Iteration loop for the MNIST step: parity of the fp32 step, stage stamps (tl variant, if
# shipped), and the plain and driver-form bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_golden.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 || { tail -30 gpurun_out/iter_tests.log; exit 1; }
tail -1 gpurun_out/iter_tests.log
if [ -f vaeb_amd/libvaeb_hip_tl.so ]; then
  timeout -k 10 120 python3 scripts/tl_stages.py > gpurun_out/tl_stages.txt 2>&1 || { tail -20 gpurun_out/tl_stages.txt; exit 1; }
fi
for i in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/bench_plain_$i.json 2> gpurun_out/bench_plain.err || { tail -20 gpurun_out/bench_plain.err; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_driver_$i.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
done
python3 -c "
import json
for f in ('bench_plain_1','bench_driver_1','bench_plain_2','bench_driver_2'):
    d=json.load(open('gpurun_out/%s.json'%f)); print(f, round(d['ms_per_step']*1000,2), 'us/step', {k: round(v*1000,2) for k,v in d['kernels_ms'].items()})"
