# Round 6: kernel-trace stats of the config-5 step with bf16 and with fp16 operands -> gpurun_out/r6sp/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6sp
mkdir -p $O
for dt in bf16 fp16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$dt -o run -- python3 bench.py --config synth --dtype $dt --steps 60 --warmup 5 --no-cpu-baseline > $O/bench_$dt.json 2> $O/err_$dt.txt || { tail $O/err_$dt.txt; exit 1; }
  cp $O/$dt/run_kernel_stats.csv $O/stats_$dt.csv
  echo "== $dt"; cut -d, -f1-8 $O/stats_$dt.csv | cut -c1-200 | head -16
done
