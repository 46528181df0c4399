# Round 5 evidence on the committed build: the full GPU suite, smoke(), driver-form (20 / 5) and
# 2000-step MNIST lines, then scripts/gpu_evidence.sh (kernel-trace stats, FETCH / WRITE and
# MFMA-busy PMC passes, bench lines with the CPU baseline) for $CONFIGS into profiles/r5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ev
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
  tail -2 $O/gpu_tests.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit 1; }
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/driver_$i.json'));print('driver form', round(d['ms_per_step']*1000,2))"
done
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/mnist_2000.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "import json;d=json.load(open('$O/mnist_2000.json'));print('2000 steps', round(d['ms_per_step']*1000,2))"
ROUND=r5 CONFIGS="${CONFIGS:-mnist frey fv fvs}" bash scripts/gpu_evidence.sh
