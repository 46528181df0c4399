# Round 5: full GPU suite, smoke(), then driver-form (20 / 5) bench lines and a 2000-step line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_$i.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
done
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/b2000.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 - <<'PY'
import json
for f in ["driver_1", "driver_2", "driver_3", "b2000"]:
    d = json.load(open(f"gpurun_out/r5check/{f}.json"))
    print(f, round(d["ms_per_step"] * 1000, 2), {k: round(v * 1000, 2) for k, v in d["kernels_ms"].items()})
PY
