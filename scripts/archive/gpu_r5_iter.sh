# Round 5 iteration: the step parity tests, then alternating A/B bench lines of one switch
# (default form vs $AB=0), 2000-step and driver-form (20 / 5).  Usage: AB=VAEB_DHD2 bash scripts/gpu_r5_iter.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5iter
mkdir -p $O
AB=${AB:-VAEB_DHD2}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_step.py} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit 1; }
for rep in 1 2; do
  for v in ${AB_VALS:-1 0}; do
    env $AB=$v timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/b_${v}_$rep.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    env $AB=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/d_${v}_$rep.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  done
done
python3 - <<PY
import json, glob
for f in sorted(glob.glob("$O/[bd]_*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], round(d["ms_per_step"] * 1000, 2), {k: round(v * 1000, 2) for k, v in d["kernels_ms"].items()})
PY
