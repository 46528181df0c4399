# Round 2: bf16 engine, weight gradients forked on a second stream after dhd (default) vs
# the fused dhd | dW2 grid (VAEB_BF_FORK=0); VAEB_BF_W3_256=0: dW3 on 256 x 128 tiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fork
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_golden.py tests/test_gpu_dropin.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/fork/pytest.log 2>&1 || { tail -30 gpurun_out/fork/pytest.log; exit 1; }
tail -1 gpurun_out/fork/pytest.log
for r in 1 2; do
for v in "1 1" "1 0" "0 1"; do
  set -- $v
  VAEB_BF_FORK=$1 VAEB_BF_W3_256=$2 timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/fork/s.json 2> gpurun_out/fork/s.err || { tail -5 gpurun_out/fork/s.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fork/s.json'));print('fork=$1 w3_256=$2', round(d['ms_per_step']*1000,1), 'us', d['elbo'])"
done
done
