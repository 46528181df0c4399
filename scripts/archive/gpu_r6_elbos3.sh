# Round 6 A/B: config 5, the ELBO stage-1 partials first on the second stream (bias_opt waits for them)

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6es
mkdir -p $O
VAEB_LIB_VARIANT=elbos3 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for v in base elbos3; do
    if [ $v = base ]; then unset VAEB_LIB_VARIANT; else export VAEB_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > $O/s_${v}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/s_${v}_$r.json'));print('$v $r', round(d['ms_per_step']*1000,1))"
  done
done
