# Round 6 A/B: config 5's Bernoulli decoder epilogue expanding its x tile from a bit copy of the
# (binary) dataset against the 16-bit tile (VAEB_LIB_VARIANT=base: the build before)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6xb
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export VAEB_LIB_VARIANT=base; else unset VAEB_LIB_VARIANT; fi
    timeout -k 10 200 python3 bench.py --config synth --steps 100 --warmup 10 --no-cpu-baseline > $O/s_${v}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/s_${v}_$r.json'));print('$v $r', round(d['ms_per_step']*1000,1), {k: round(x*1000,1) for k, x in d.get('kernels_ms', {}).items() if k in ('bf_decout',)})"
  done
done
for v in base new; do
  if [ $v = base ]; then export VAEB_LIB_VARIANT=base; else unset VAEB_LIB_VARIANT; fi
  timeout -k 10 200 python3 bench.py --config synth --dtype bf16 --steps 100 --warmup 10 --no-cpu-baseline > $O/b_${v}.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_${v}.json'));print('bf16 $v', round(d['ms_per_step']*1000,1), {k: round(x*1000,1) for k, x in d.get('kernels_ms', {}).items() if k in ('bf_decout',)})"
done
