# Encoder hand-off moved into the decoder launch (VAEB_ENC_RED=1): parity under the mode,
# the mode-agreement test, MNIST / Frey A/B (interleaved) and the stage timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/red
timeout -k 10 500 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_golden.py tests/test_gpu_api.py tests/test_gpu_pins.py tests/test_gpu_dropin.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/red/pytest.log 2>&1 || { tail -40 gpurun_out/red/pytest.log; exit 1; }
tail -1 gpurun_out/red/pytest.log
for r in 1 2; do
for v in 0 1; do
  VAEB_ENC_RED=$v timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/red/m$v.json 2> gpurun_out/red/m$v.err || { tail -5 gpurun_out/red/m$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/red/m$v.json'));print('mnist red=$v', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
  VAEB_ENC_RED=$v timeout -k 10 120 python3 bench.py --config frey --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/red/f$v.json 2> gpurun_out/red/f$v.err || { tail -5 gpurun_out/red/f$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/red/f$v.json'));print('frey red=$v', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
done
done
VAEB_ENC_RED=1 timeout -k 10 120 python3 scripts/tl_stages.py > gpurun_out/red/tl.txt 2>&1 || exit 1
head -24 gpurun_out/red/tl.txt
