# Round 2: bf16 engine with dhd + dW2 in one grid -- bf16 parity tests, then synth bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/envab
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_bf.log 2>&1 || { tail -30 gpurun_out/pytest_bf.log; exit 1; }
tail -1 gpurun_out/pytest_bf.log
for r in 1 2; do
  for v in 1 0; do
    VAEB_BF_FUSE=$v timeout -k 10 200 python3 bench.py --config synth --no-cpu-baseline > gpurun_out/envab/b$v.json 2> gpurun_out/envab/b$v.err || { tail -5 gpurun_out/envab/b$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/envab/b$v.json'));print('fuse=$v', round(d['ms_per_step']*1000,1), 'us', {k: round(x*1000,1) for k,x in d['kernels_ms'].items()}, d['roofline']['kernel'], round(d['roofline']['frac'],3))"
  done
done
