# Config 5 (synthetic 4096-2048-128, B=8192, bf16): bench line + kernel-trace profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/synth
mkdir -p $O
timeout -k 10 300 python3 bench.py --config synth > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-2500 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config synth --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err || exit 1
cut -c1-220 $O/trace/run_kernel_stats.csv
