# Config-5 GEMM diagnostics: stall / LDS-conflict / MFMA-busy counters per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/synth_pmc
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o run -- python3 bench.py --config synth --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/p1.err || { tail -5 $O/p1.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA --output-format csv -d $O/p2 -o run -- python3 bench.py --config synth --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
python3 scripts/pmc_summary.py $O/pmc.json $O/p1 $O/p2 > /dev/null
python3 - <<'PY'
import json
d = json.load(open('gpurun_out/synth_pmc/pmc.json'))
for k, v in d.items():
    if 'gemm_kernel' not in k: continue
    print(k[40:110])
    print('   ', {c: round(x) for c, x in v.items() if c != 'launches'})
PY
