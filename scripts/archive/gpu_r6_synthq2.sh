# Round 6: config-5 (fp16) step timeline per hardware queue from a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6sq2
mkdir -p $O
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config synth --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/line.json 2> $GRAFT_REPO_ROOT/$O/err.txt || { tail $GRAFT_REPO_ROOT/$O/err.txt; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/step_queues.py $O/kt/run_kernel_trace.csv > $O/queues.txt || exit 1
cat $O/queues.txt
