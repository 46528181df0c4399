# Encoder column tiles per workgroup: parity at VAEB_ENC_CT=4, then the MNIST A/B 1 / 2 / 4
# (interleaved rounds) and the stage timeline at 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ct
VAEB_ENC_CT=4 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_step.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/ct/tests.log 2>&1 || { tail -30 gpurun_out/ct/tests.log; exit 1; }
tail -2 gpurun_out/ct/tests.log
for r in 1 2; do
  for v in 1 2 4; do
    VAEB_ENC_CT=$v timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/ct/v$v.json 2> gpurun_out/ct/v$v.err || { tail -5 gpurun_out/ct/v$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ct/v$v.json'));print('CT=$v', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
  done
done
VAEB_ENC_CT=4 timeout -k 10 120 python3 scripts/tl_stages.py > gpurun_out/ct/tl4.txt 2>&1 || exit 1
head -12 gpurun_out/ct/tl4.txt
