# bf16 engine: its GPU tests, then alternating config-5 bench lines per setting.
# Usage: bash scripts/gpu_r3_bfab.sh "VAR=a" "VAR=b" ...   (BENCH_ARGS overrides the run length)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_golden.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bf_tests.log 2>&1 || { tail -40 gpurun_out/bf_tests.log; exit 1; }
tail -1 gpurun_out/bf_tests.log
: > gpurun_out/bfab.txt
for rep in 1 2; do
  for setting in "$@"; do
    env $setting timeout -k 10 200 python3 bench.py --config synth --no-cpu-baseline ${BENCH_ARGS:---steps 300 --warmup 30} > gpurun_out/bfab_line.json 2> gpurun_out/bfab.err || { tail -20 gpurun_out/bfab.err; exit 1; }
    python3 -c "
import json,sys
d=json.load(open('gpurun_out/bfab_line.json')); print(sys.argv[1], round(d['ms_per_step']*1000,2), 'us/step', {k: round(v*1000,2) for k,v in d['kernels_ms'].items()})" "$setting" | tee -a gpurun_out/bfab.txt
  done
done
