# Round 4 final check: the full GPU suite, smoke(), a driver-form bench line and the last
# launch's stage stamps on the committed build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/driver_form.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_form.json'));print('driver form', round(d['ms_per_step']*1000,2), d['roofline']['kernel'], round(d['roofline']['frac'],4))"
timeout -k 10 120 python3 scripts/tl_dump.py mnist > /dev/null && python3 scripts/tl_last.py > $O/tl_last.txt && timeout -k 10 120 python3 scripts/tl_stages.py > $O/tl_stages.txt || exit 1
head -4 $O/tl_last.txt
