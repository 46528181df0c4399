# Round 6 A/B: the 8-phase loop with two counted waits per K-tile (phase 0: vmcnt(6), phase 3:
# vmcnt(8)) instead of one per phase (VAEB_LIB_VARIANT=w2 against the product build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6w2
mkdir -p $O
export VAEB_LIB_VARIANT=w2
timeout -k 10 300 python3 scripts/gemm8_screen.py 150 > $O/screen.txt 2>&1; rc=$?; tail -2 $O/screen.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in base w2; do
    if [ $v = w2 ]; then export VAEB_LIB_VARIANT=w2; else unset VAEB_LIB_VARIANT; fi
    timeout -k 10 120 python3 scripts/gemm_vs_blas.py fp16 > $O/blas_${v}_$r.txt 2>&1 || { tail $O/blas_${v}_$r.txt; exit 1; }
    echo "== $v $r"; grep "M=" $O/blas_${v}_$r.txt | sed 's/hipBLASLt.*//' | cut -c1-110
  done
done
for r in 1 2 3; do
  for v in base w2; do
    if [ $v = w2 ]; then export VAEB_LIB_VARIANT=w2; else unset VAEB_LIB_VARIANT; fi
    timeout -k 10 200 python3 bench.py --config synth --steps 100 --warmup 10 --no-cpu-baseline > $O/s_${v}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/s_${v}_$r.json'));print('$v $r', round(d['ms_per_step']*1000,1), {k: round(v*1000,1) for k, v in d.get('kernels_ms', {}).items() if k in ('bf_enc','bf_decout','bf_dhd_dW26','bf_dW3')})"
  done
done
