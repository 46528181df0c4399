# Round 2: encoder with two 16-column h tiles per workgroup (VAEB_ENC_CT=2: half the
# contributors per latent element) vs one; slabs (MNIST) and atomics (Frey).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/encct
VAEB_ENC_CT=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/encct/pytest.log 2>&1 || { tail -40 gpurun_out/encct/pytest.log; exit 1; }
tail -1 gpurun_out/encct/pytest.log
for r in 1 2; do
for v in 1 2; do
  for cfg in mnist frey fv; do
    VAEB_ENC_CT=$v timeout -k 10 120 python3 bench.py --config $cfg --steps 4000 --warmup 200 --no-cpu-baseline > gpurun_out/encct/$cfg$v.json 2> gpurun_out/encct/$cfg$v.err || { tail -5 gpurun_out/encct/$cfg$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/encct/$cfg$v.json'));print('$cfg ct=$v', round(d['ms_per_step']*1000,2), {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
  done
done
done
