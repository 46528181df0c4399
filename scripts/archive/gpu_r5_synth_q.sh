# Round 5: kernel trace of the config-5 forked step under VAEB_BF_FORKPT=$FP (which HW queue each
# launch of the graph ran on, per-step anatomy), then bench lines alternating FORKPT 1 / $FP.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
for fp in 1 ${FP:-0}; do
  VAEB_BF_FORKPT=$fp timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$fp -o run -- python3 bench.py --config synth --steps 12 --warmup 3 --no-cpu-baseline > $O/line_$fp.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 scripts/step_queues.py $O/tr_$fp/run_kernel_trace.csv > $O/queues_$fp.txt || exit 1
  head -24 $O/queues_$fp.txt
done
