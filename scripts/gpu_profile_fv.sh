# Config-4 evidence (literal FV and the weight-sampling FVS extension): kernel-trace stats,
# FETCH_SIZE / WRITE_SIZE PMC passes (separate runs), then the bench lines with the CPU
# baseline.  -> gpurun_out/round/<config>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in fv fvs; do
  O=gpurun_out/round/$cfg
  mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config $cfg --steps 1000 --warmup 100 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err || { tail $O/bench_trace.err; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline > /dev/null 2> $O/fetch.err || { tail $O/fetch.err; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline > /dev/null 2> $O/write.err || { tail $O/write.err; exit 1; }
  python3 scripts/pmc_summary.py $O/pmc_per_launch.json $O/fetch $O/write > $O/pmc_summary.txt || exit 1
  cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv
  cp $O/pmc_per_launch.json profiles/r1/pmc_${cfg}_per_launch.json
  timeout -k 10 200 python3 bench.py --config $cfg > $O/bench_line.json 2> $O/bench_line.err || { tail $O/bench_line.err; exit 1; }
  echo "== $cfg"; cut -c1-150 $O/kernel_stats.csv | head -12; cut -c1-400 $O/bench_line.json
done
