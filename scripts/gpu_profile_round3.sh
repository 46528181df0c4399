# Round evidence: per config (mnist, frey, synth) a kernel-trace + stats profile and the
# FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, MI355X_MICROARCH.md §HBM), folded
# per launch by scripts/pmc_summary.py.  -> gpurun_out/round3/<config>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in mnist frey fv fvs synth; do
  O=gpurun_out/round3/$cfg
  mkdir -p $O
  if [ $cfg = synth ]; then S="--steps 30 --warmup 3"; P="--steps 10 --warmup 2"; else S="--steps 1000 --warmup 100"; P="--steps 200 --warmup 20"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config $cfg $S --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err || { tail $O/bench_trace.err; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --config $cfg $P --no-cpu-baseline > /dev/null 2> $O/fetch.err || { tail $O/fetch.err; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --config $cfg $P --no-cpu-baseline > /dev/null 2> $O/write.err || { tail $O/write.err; exit 1; }
  python3 scripts/pmc_summary.py $O/pmc_per_launch.json $O/fetch $O/write > $O/pmc_summary.txt || exit 1
  cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv
  echo "== $cfg"; cut -c1-150 $O/kernel_stats.csv | head -12
done
