# Round 2: per-group 16-byte panel loads in the last weight-gradient launch (Frey: the dW3
# group keeps vector loads although dW1 / dW4|dW5 cannot) vs all-or-nothing.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gvec
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gvec/pytest.log 2>&1 || { tail -40 gpurun_out/gvec/pytest.log; exit 1; }
tail -1 gpurun_out/gvec/pytest.log
for r in 1 2; do
for v in 1 0; do
  for cfg in frey mnist; do
    VAEB_W3_GVEC=$v timeout -k 10 120 python3 bench.py --config $cfg --steps 4000 --warmup 200 --no-cpu-baseline > gpurun_out/gvec/$cfg$v.json 2> gpurun_out/gvec/$cfg$v.err || { tail -5 gpurun_out/gvec/$cfg$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/gvec/$cfg$v.json'));print('$cfg gvec=$v', round(d['ms_per_step']*1000,2), {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
  done
done
done
