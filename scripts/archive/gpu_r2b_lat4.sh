# bf16 engine: 16-byte latent kernels (VAEB_BF_LAT4) and the side-stream ELBO partials:
# bf16 parity tests, then config-5 A/B (interleaved).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lat4
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_golden.py tests/test_gpu_dropin.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/lat4/pytest.log 2>&1 || { tail -30 gpurun_out/lat4/pytest.log; exit 1; }
tail -1 gpurun_out/lat4/pytest.log
for r in 1 2; do
for v in 1 0; do
  VAEB_BF_LAT4=$v timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/lat4/s$v.json 2> gpurun_out/lat4/s$v.err || { tail -5 gpurun_out/lat4/s$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/lat4/s$v.json'));print('lat4=$v', round(d['ms_per_step']*1000,1), 'us', d['elbo'], {k: round(x*1000,1) for k,x in d['kernels_ms'].items()})"
done
done
