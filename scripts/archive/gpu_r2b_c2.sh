# Bernoulli decoder with two 16-column tiles per workgroup (VAEB_DECOUT_C2): parity under
# the mode, MNIST A/B (interleaved), stage timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c2
VAEB_DECOUT_C2=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_golden.py tests/test_gpu_api.py tests/test_gpu_dropin.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/c2/pytest.log 2>&1 || { tail -40 gpurun_out/c2/pytest.log; exit 1; }
tail -1 gpurun_out/c2/pytest.log
for r in 1 2; do
for v in 0 1; do
  VAEB_DECOUT_C2=$v timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/c2/m$v.json 2> gpurun_out/c2/m$v.err || { tail -5 gpurun_out/c2/m$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c2/m$v.json'));print('mnist c2=$v', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
  VAEB_DECOUT_C2=$v VAEB_ENC_RED=0 timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/c2/n$v.json 2> gpurun_out/c2/n$v.err || { tail -5 gpurun_out/c2/n$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c2/n$v.json'));print('mnist red=0 c2=$v', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
done
done
