# Round 2: atomic hand-offs at fan-in <= 16 (default) -- GPU suite, then per-config bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/atomic
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/atomic/pytest2.log 2>&1 || { tail -40 gpurun_out/atomic/pytest2.log; exit 1; }
tail -1 gpurun_out/atomic/pytest2.log
for cfg in mnist frey fv fvs; do
  timeout -k 10 120 python3 bench.py --config $cfg --steps 2000 --warmup 200 --no-cpu-baseline > gpurun_out/atomic/b_$cfg.json 2> gpurun_out/atomic/b_$cfg.err || { tail -5 gpurun_out/atomic/b_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/atomic/b_$cfg.json'));print('$cfg', round(d['ms_per_step']*1000,2), {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
done
