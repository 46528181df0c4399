# Round 3: world-1 DP cost on both engines (dp_world1_timing), current build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/dp_world1_timing.py > gpurun_out/dp_world1.txt 2>&1 || { tail -20 gpurun_out/dp_world1.txt; exit 1; }
grep "us/step" gpurun_out/dp_world1.txt
timeout -k 10 400 python3 scripts/dp_world1_timing.py --bf16 > gpurun_out/dp_world1_bf16.txt 2>&1 || { tail -20 gpurun_out/dp_world1_bf16.txt; exit 1; }
grep "us/step" gpurun_out/dp_world1_bf16.txt | cut -c1-200
