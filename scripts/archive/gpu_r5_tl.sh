# Round 5 timeline: per-workgroup stage stamps (VAEB_TIMELINE build, libvaeb_hip_tl.so) of the
# default step and of $AB=0, dumped for offline analysis plus the per-launch stage summary.
# (libvaeb_hip_tl.so is listed in .gpurunignore except for these runs.)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5tl
mkdir -p $O
AB=${AB:-VAEB_DHD2}
for v in 1 0; do
  env $AB=$v TL_SUFFIX=_$v timeout -k 10 120 python3 scripts/tl_dump.py mnist > /dev/null || exit 1
  env $AB=$v timeout -k 10 120 python3 scripts/tl_stages.py > $O/stages_$v.txt || exit 1
done
mv gpurun_out/tl_mnist_*.npz $O/
head -60 $O/stages_1.txt
