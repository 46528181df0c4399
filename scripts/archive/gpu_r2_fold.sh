# Round 2: folded latent backward -- full GPU suite, then A/B against the P67 launch
# (VAEB_FOLD_BWD=0) on MNIST and Frey shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest.log
tail -3 gpurun_out/pytest.log
grep -E "FAILED|ERROR" gpurun_out/pytest.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
mkdir -p gpurun_out/envab
for cfg in mnist frey; do
for r in 1 2; do
  for v in 1 0; do
    VAEB_FOLD_BWD=$v timeout -k 10 120 python3 bench.py --config $cfg --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/envab/f$v.json 2> gpurun_out/envab/f$v.err || { tail -5 gpurun_out/envab/f$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/envab/f$v.json'));print('$cfg fold=$v', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()}, 'elbo', round(d['elbo'],4))"
  done
done
done
