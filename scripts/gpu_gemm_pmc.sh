# The 8-phase GEMM against hipBLASLt, counter by counter (scripts/gemm_pmc_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gemm_pmc
mkdir -p $O
P="python3 scripts/gemm_pmc_probe.py fp16"
timeout -k 10 120 $P > $O/plain.txt 2>&1 || { tail $O/plain.txt; exit 1; }
cat $O/plain.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $P > /dev/null 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d $O/p1 -o run -- $P > /dev/null 2> $O/p1.err || { tail -5 $O/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- $P > /dev/null 2> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/p3 -o run -- $P > /dev/null 2> $O/p3.err || { tail -5 $O/p3.err; exit 1; }
python3 scripts/pmc_summary.py $O/pmc.json $O/p1 $O/p2 $O/p3 > /dev/null || exit 1
python3 - <<'PY'
import json, csv, glob
d = json.load(open('gpurun_out/gemm_pmc/pmc.json'))
for k, v in sorted(d.items()):
    if v.get('launches', 0) < 5: continue
    print(k[:100])
    print('   ', {c: round(x) for c, x in v.items()})
for p in glob.glob('gpurun_out/gemm_pmc/kt/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        print(r['Name'][:90], r['Calls'], r['AverageNs'])
PY
