# Round 5: kernel trace of the config-5 (bf16, 4096-2048-128, B = 8192) forked step, per-position
# anatomy (scripts/dp_fork_anatomy.py keyed on the encoder GEMM).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5synth
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --config synth --steps 12 --warmup 3 --no-cpu-baseline > $O/line.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r5synth/tr/run_kernel_trace.csv")))
from collections import Counter
print(Counter(r["Kernel_Name"].split("(")[0][:90] for r in rows).most_common(40))
PY
