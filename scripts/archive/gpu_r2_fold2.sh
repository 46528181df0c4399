set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/envab
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_dropin.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_fold.log 2>&1 || { tail -30 gpurun_out/pytest_fold.log; exit 1; }
tail -1 gpurun_out/pytest_fold.log
for r in 1 2; do
  for v in 1 0; do
    VAEB_FOLD_BWD=$v timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/envab/f$v.json 2> gpurun_out/envab/f$v.err || { tail -5 gpurun_out/envab/f$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/envab/f$v.json'));print('fold=$v', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
  done
done
timeout -k 10 100 python3 scripts/tl_stages.py > gpurun_out/tl_stages.txt 2>&1
head -75 gpurun_out/tl_stages.txt
