# Round 6 A/B: the 16-byte (LDS-transposed) Adagrad epilogue of the 256-wide weight-gradient tiles
# against the per-element form (VAEB_LIB_VARIANT=base: the build before)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6av
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_bf16.py tests/test_gpu_dp_ranks.py tests/test_gpu_cli_dp.py tests/test_gpu_dropin.py tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export VAEB_LIB_VARIANT=base; else unset VAEB_LIB_VARIANT; fi
    timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > $O/s_${v}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/s_${v}_$r.json'));print('$v $r', round(d['ms_per_step']*1000,1))"
  done
done
