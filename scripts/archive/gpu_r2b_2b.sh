# bf16 engine: bias sums with segment-uniform blocks; enc / forked dhd on 256 x 128 tiles,
# two blocks per CU (VAEB_BF_ENC2B, VAEB_BF_DHD2B): parity, then config-5 A/B (interleaved).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/b2
VAEB_BF_ENC2B=1 VAEB_BF_DHD2B=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_golden.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/b2/pytest2.log 2>&1 || { tail -30 gpurun_out/b2/pytest2.log; exit 1; }
tail -1 gpurun_out/b2/pytest2.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_golden.py tests/test_gpu_dropin.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/b2/pytest.log 2>&1 || { tail -30 gpurun_out/b2/pytest.log; exit 1; }
tail -1 gpurun_out/b2/pytest.log
for r in 1 2; do
for v in "0 0" "1 0" "0 1" "1 1"; do
  set -- $v
  VAEB_BF_ENC2B=$1 VAEB_BF_DHD2B=$2 timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/b2/s.json 2> gpurun_out/b2/s.err || { tail -5 gpurun_out/b2/s.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b2/s.json'));print('enc2b=$1 dhd2b=$2', round(d['ms_per_step']*1000,1), 'us', d['elbo'], 'bias', round(d['kernels_ms']['bf_bias_elbo']*1000,1))"
done
done
