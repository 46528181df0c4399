# bf16 engine: dz split-K at >= 16 K tiles per slice (default now 4 at config 5) vs 8
# (VAEB_BF_KS_DZ=8): bf16 parity, then interleaved config-5 runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dz
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_golden.py tests/test_gpu_dropin.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/dz/pytest.log 2>&1 || { tail -30 gpurun_out/dz/pytest.log; exit 1; }
tail -1 gpurun_out/dz/pytest.log
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/dz/s.json 2> gpurun_out/dz/s.err || { tail -5 gpurun_out/dz/s.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/dz/s.json'));print('default', round(d['ms_per_step']*1000,1), 'us')"
  VAEB_BF_KS_DZ=8 timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/dz/s.json 2> gpurun_out/dz/s.err || { tail -5 gpurun_out/dz/s.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/dz/s.json'));print('ks_dz=8', round(d['ms_per_step']*1000,1), 'us')"
done
