# Config-5 (bf16) kernel trace of the default (forked) step: the last step's launches as a
# timeline with queue ids.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tr5
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr5/raw -o run -- python3 bench.py --config synth --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/tr5/bench.json 2> gpurun_out/tr5/bench.err || { tail -5 gpurun_out/tr5/bench.err; exit 1; }
python3 scripts/trace_timeline.py gpurun_out/tr5/raw 40 > gpurun_out/tr5/timeline.txt
cat gpurun_out/tr5/timeline.txt
