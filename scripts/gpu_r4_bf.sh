# Round 4, config 5: the two-slice weight gradients -- parity tests, bare GEMMs against
# hipBLASLt, then interleaved 300-step synth benches with VAEB_BF_SPLIT2=0 / 1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/bf
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_bf16.py \
  -k "two_slices or split2 or gemm8 or forked or dp_path" > gpurun_out/bf/tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/bf/tests.log | head -20; tail -5 gpurun_out/bf/tests.log; exit 1; }
tail -2 gpurun_out/bf/tests.log
timeout -k 10 300 python3 scripts/gemm_vs_blas.py > gpurun_out/bf/gemm.txt 2>&1 || { tail gpurun_out/bf/gemm.txt; exit 1; }
cat gpurun_out/bf/gemm.txt
for r in 1 2; do
  for v in 0 1; do
    VAEB_BF_SPLIT2=$v timeout -k 10 300 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/bf/s$v.json 2> gpurun_out/bf/s$v.err || { tail gpurun_out/bf/s$v.err; exit 1; }
    cp gpurun_out/bf/s$v.json gpurun_out/bf/s${v}_r$r.json
    python3 -c "import json;d=json.load(open('gpurun_out/bf/s$v.json'));print('split2=$v', round(d['ms_per_step']*1000,1), 'us/step')"
  done
done
