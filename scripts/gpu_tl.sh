# In-kernel timeline only.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/gpu_timeline.py > gpurun_out/timeline.txt 2>&1
