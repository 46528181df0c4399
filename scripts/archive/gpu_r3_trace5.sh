# Config-5 forked step as a kernel-trace timeline (last step's launches with queue ids).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tr5
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr5/raw -o run -- python3 scripts/synth_steps.py 8 > gpurun_out/tr5/run.log 2>&1 || { tail -5 gpurun_out/tr5/run.log; exit 1; }
python3 scripts/trace_timeline.py gpurun_out/tr5/raw 40 > gpurun_out/tr5/timeline.txt
cat gpurun_out/tr5/timeline.txt
