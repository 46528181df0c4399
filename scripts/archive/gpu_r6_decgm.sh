# Round 6 A/B: the two-tile MNIST decoder's tile order -- runs of GM row blocks sweep the column
# tiles (GM 1 = row-major, the default; 4 ~ a 2 x 4 row x column split of the XCDs; 7 = column-major)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6gm
mkdir -p $O
us() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['ms_per_step']*1000,2), 'us/step')"; }
VAEB_DEC_GM=4 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_step.py -x -q --timeout 120 --timeout-method thread \
  -k "atomic_and_slab or mnist" > $O/tests_gm4.txt 2>&1 || { tail -30 $O/tests_gm4.txt; exit 1; }
tail -1 $O/tests_gm4.txt
for r in 1 2; do
  for gm in 1 2 4 7; do
    VAEB_DEC_GM=$gm timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/m2000_${gm}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    us $O/m2000_${gm}_$r.json "2000 gm$gm $r"
  done
done
cd /tmp
for gm in 1 2 4 7; do
  VAEB_DEC_GM=$gm timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt$gm -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 500 --warmup 50 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  VAEB_DEC_GM=$gm timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pf$gm -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  VAEB_DEC_GM=$gm timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pw$gm -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > /dev/null 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for gm in 1 2 4 7; do
  python3 scripts/pmc_summary.py $O/pmc$gm.json $O/pf$gm $O/pw$gm > /dev/null || exit 1
  python3 - $gm <<'PY'
import json, csv, glob, sys
gm = sys.argv[1]
d = json.load(open(f'gpurun_out/r6gm/pmc{gm}.json'))
for k, v in d.items():
    if 'decout_z2' in k:
        print('gm', gm, 'decout_z2 MB/launch', round(v['hbm_bytes_per_launch'] / 1e6, 2))
for p in glob.glob(f'gpurun_out/r6gm/kt{gm}/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        if 'vaeb' in r['Name'] and int(r['Calls']) > 100:
            print('gm', gm, r['Name'][:60], r['AverageNs'])
PY
done
timeout -k 10 200 python3 scripts/call_anatomy.py > gpurun_out/r6gm/call_anatomy.txt 2>&1 || exit 1; cat gpurun_out/r6gm/call_anatomy.txt
