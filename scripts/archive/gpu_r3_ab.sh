# A/B of library switches on the MNIST step: parity of the fp32 step, then alternating
# 2000-step bench lines per setting.  Usage: bash scripts/gpu_r3_ab.sh "VAR=a" "VAR=b" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_golden.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
: > gpurun_out/ab.txt
for rep in 1 2 3; do
  for setting in "$@"; do
    env $setting timeout -k 10 200 python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_line.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python3 -c "
import json,sys
d=json.load(open('gpurun_out/ab_line.json')); print(sys.argv[1], round(d['ms_per_step']*1000,2), 'us/step', {k: round(v*1000,2) for k,v in d['kernels_ms'].items()})" "$setting" | tee -a gpurun_out/ab.txt
  done
done
