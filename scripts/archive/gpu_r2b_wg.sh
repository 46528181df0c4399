# Weight-gradient tiles: LDS -> MFMA loop unrolled over the stage's chunks.  fp32 parity
# (step, golden, AE, drop-in), then MNIST / Frey / FV bench lines and the stage timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/wg
timeout -k 10 500 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_golden.py tests/test_gpu_ae.py tests/test_gpu_dropin.py tests/test_gpu_api.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/wg/pytest.log 2>&1 || { tail -40 gpurun_out/wg/pytest.log; exit 1; }
tail -1 gpurun_out/wg/pytest.log
for r in 1 2; do
for c in mnist frey fv; do
  timeout -k 10 120 python3 bench.py --config $c --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/wg/$c.json 2> gpurun_out/wg/$c.err || { tail -5 gpurun_out/wg/$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/wg/$c.json'));print('$c', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
done
done
timeout -k 10 120 python3 scripts/tl_stages.py > gpurun_out/wg/tl.txt 2>&1 || exit 1
sed -n 20,50p gpurun_out/wg/tl.txt
