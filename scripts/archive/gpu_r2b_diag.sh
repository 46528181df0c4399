# Driver-form first-call cost with / without hipGraphUpload, and the MNIST stage timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for u in 0 1 0 1; do
  VAEB_GRAPH_UPLOAD=$u timeout -k 10 120 python3 scripts/first_call.py >> gpurun_out/first_call.txt 2>&1 || exit 1
done
cat gpurun_out/first_call.txt
timeout -k 10 120 python3 scripts/tl_stages.py > gpurun_out/tl_stages.txt 2>&1 || exit 1
head -60 gpurun_out/tl_stages.txt
