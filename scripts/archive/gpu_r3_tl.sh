# In-kernel stage stamps of the MNIST step (needs vaeb_amd/libvaeb_hip_tl.so, built here).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/tl_stages.py > gpurun_out/tl_stages.txt 2>&1 && \
timeout -k 10 120 python3 scripts/gpu_timeline2.py > gpurun_out/timeline2.txt 2>&1
rc=$?; tail -5 gpurun_out/tl_stages.txt; exit $rc
