# Round profile of the MNIST step: kernel trace + stats, then the HBM-traffic PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md) and one SQ pass,
# folded per launch by scripts/pmc_summary.py.  Output: gpurun_out/prof_r1/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_r1
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_fetch.json 2> $O/bench_fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_write.json 2> $O/bench_write.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $O/insts -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_insts.json 2> $O/bench_insts.err || exit 1
python3 scripts/pmc_summary.py $O/pmc_per_launch.json $O/fetch $O/write $O/insts
cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv
cut -c1-200 $O/kernel_stats.csv
