# Round 3: config 5 with the 8-phase 256^2 GEMMs per layout pair (VAEB_BF_GEMM8 bit mask:
# 2 KC x KO (enc), 1 KC x KC (dhd), 8 KO x KO (dW2 / dW3)) against the BK = 32 ring.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
VAEB_BF_GEMM8=15 timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bf16_g8_tests.log 2>&1; rc=$?
tail -2 gpurun_out/bf16_g8_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/bf16_g8_tests.log | head -30; exit 1; }
for r in 1 2; do for g in 0 2 3 10 11; do
  VAEB_BF_GEMM8=$g timeout -k 10 300 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/synth_g${g}_$r.json 2> gpurun_out/synth.err || { tail -20 gpurun_out/synth.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/synth_g${g}_$r.json')); k=d['kernels_ms']
print('gemm8 mask $g run $r', round(d['ms_per_step']*1000,1), 'us/step', {x: round(v*1000,1) for x,v in k.items() if v > 0.09})"
done; done
