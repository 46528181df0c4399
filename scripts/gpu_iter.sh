# Iteration check: the full GPU parity suite, then MNIST and Frey bench lines (no CPU leg).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/iter
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter/tests.log 2>&1 || { tail -30 gpurun_out/iter/tests.log; exit 1; }
tail -2 gpurun_out/iter/tests.log
for cfg in mnist frey; do
  timeout -k 10 120 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/iter/$cfg.json 2> gpurun_out/iter/$cfg.err || { tail -5 gpurun_out/iter/$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/iter/$cfg.json'));print('$cfg', round(d['ms_per_step']*1000,2), 'us', round(d['value']/1e6,3), 'M img/s', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
done
