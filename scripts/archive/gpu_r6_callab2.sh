# Round 6 A/B: update_many's short call -- the order uploaded before the eager first step and
# one graph family per starting arena (new) against the round-5 call (VAEB_LIB_VARIANT=base)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6cab2
mkdir -p $O
us() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['ms_per_step']*1000,2), 'us/step')"; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_api.py tests/test_gpu_dropin.py tests/test_gpu_step.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export VAEB_LIB_VARIANT=base; else unset VAEB_LIB_VARIANT; fi
    timeout -k 10 120 python3 scripts/call_ab2.py 2>&1 | grep "call:" || exit 1
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_${v}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    us $O/driver_${v}_$r.json "driver $v $r"
  done
done
unset VAEB_LIB_VARIANT
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/scripts/call_trace.py 20 > $GRAFT_REPO_ROOT/$O/call_trace.txt 2>&1 || exit 1
