# Kernel-preamble change (no implicit-argument / debug-pointer loads ahead of the operand
# loads) + bf16 16-byte latent kernels: fp32 and bf16 parity, MNIST bench (long + driver
# form), config-5 A/B of VAEB_BF_LAT4, MNIST stage timeline (tl variant).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pre
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_api.py tests/test_gpu_bf16.py tests/test_gpu_golden.py tests/test_gpu_dropin.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/pre/pytest.log 2>&1 || { tail -30 gpurun_out/pre/pytest.log; exit 1; }
tail -1 gpurun_out/pre/pytest.log
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/pre/m.json 2> gpurun_out/pre/m.err || { tail -5 gpurun_out/pre/m.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/pre/m.json'));print('mnist', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/pre/d.json 2> gpurun_out/pre/d.err || { tail -5 gpurun_out/pre/d.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/pre/d.json'));print('driver form', round(d['ms_per_step']*1000,2), 'us')"
  timeout -k 10 120 python3 bench.py --config frey --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/pre/f.json 2> gpurun_out/pre/f.err || { tail -5 gpurun_out/pre/f.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/pre/f.json'));print('frey', round(d['ms_per_step']*1000,2), 'us')"
done
for r in 1 2; do
for v in 1 0; do
  VAEB_BF_LAT4=$v timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/pre/s$v.json 2> gpurun_out/pre/s$v.err || { tail -5 gpurun_out/pre/s$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/pre/s$v.json'));print('synth lat4=$v', round(d['ms_per_step']*1000,1), 'us', d['elbo'], {k: round(x*1000,1) for k,x in d['kernels_ms'].items()})"
done
done
timeout -k 10 120 python3 scripts/tl_stages.py > gpurun_out/pre/tl.txt 2>&1 || exit 1
head -48 gpurun_out/pre/tl.txt
