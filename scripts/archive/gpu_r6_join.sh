# Round 6 A/B: the 16-bit step's second stream joined at the NEXT step's heads launch (h double-
# buffered) instead of at the step's end (VAEB_LIB_VARIANT=base: the build before)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6join
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_bf16.py tests/test_gpu_dp_ranks.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export VAEB_LIB_VARIANT=base; else unset VAEB_LIB_VARIANT; fi
    timeout -k 10 200 python3 bench.py --config synth --steps 100 --warmup 10 --no-cpu-baseline > $O/s_${v}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/s_${v}_$r.json'));print('$v $r', round(d['ms_per_step']*1000,1))"
  done
done
unset VAEB_LIB_VARIANT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config synth --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> $GRAFT_REPO_ROOT/$O/kt.err || { tail $GRAFT_REPO_ROOT/$O/kt.err; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/step_queues.py $O/kt/run_kernel_trace.csv > $O/queues.txt || exit 1
cat $O/queues.txt
