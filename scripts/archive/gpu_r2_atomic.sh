# Round 2: folded latent hand-offs by counted fixed-point atomics (default) vs slabs +
# ticket + reducer (VAEB_ATOMIC_HO=0): GPU suite on the default, then MNIST / Frey A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/atomic
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/atomic/pytest.log 2>&1 || { tail -40 gpurun_out/atomic/pytest.log; exit 1; }
tail -1 gpurun_out/atomic/pytest.log
for r in 1 2; do
for v in 1 0; do
  for cfg in mnist frey; do
    VAEB_ATOMIC_HO=$v timeout -k 10 120 python3 bench.py --config $cfg --steps 4000 --warmup 200 --no-cpu-baseline > gpurun_out/atomic/$cfg$v.json 2> gpurun_out/atomic/$cfg$v.err || { tail -5 gpurun_out/atomic/$cfg$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/atomic/$cfg$v.json'));print('$cfg atomic=$v', round(d['ms_per_step']*1000,2), {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
  done
done
done
