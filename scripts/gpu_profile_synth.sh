# Config-5 profile (synthetic 4096-2048-128, B=8192, bf16 engine): bench line, kernel
# trace + stats, FETCH_SIZE / WRITE_SIZE passes (separate), SQ pass.  -> gpurun_out/prof_synth
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_synth
mkdir -p $O
timeout -k 10 300 python3 bench.py --config synth > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config synth --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --config synth --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/fetch.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --config synth --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/write.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/insts -o run -- python3 bench.py --config synth --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/insts.err || exit 1
python3 scripts/pmc_summary.py $O/pmc_per_launch.json $O/fetch $O/write $O/insts > $O/pmc_summary.txt
cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv
cut -c1-200 $O/kernel_stats.csv | head -20
cut -c1-600 $O/bench.json
