# Round 6 A/B: one graph family per starting arena (the 19 steps after update_many's eager first
# step as ONE graph) against the round-5 form (one step back to arena 0, then the arena-0 graph;
# VAEB_LIB_VARIANT=base, the previous build kept beside the new one for this run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6gf
mkdir -p $O
us() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['ms_per_step']*1000,2), 'us/step')"; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_api.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export VAEB_LIB_VARIANT=base; else unset VAEB_LIB_VARIANT; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_${v}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    us $O/driver_${v}_$r.json "driver $v $r"
  done
done
unset VAEB_LIB_VARIANT
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/m2000_new.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
us $O/m2000_new.json "2000 new"
timeout -k 10 200 python3 scripts/call_anatomy.py > $O/call_anatomy_new.txt 2>&1 || exit 1
tail -9 $O/call_anatomy_new.txt
