# A/B: forked side stream vs single stream step graphs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 bench.py --steps 4000 --warmup 200 --no-cpu-baseline > gpurun_out/ab_fork.json 2>&1 || exit 1
VAEB_SINGLE_STREAM=1 timeout -k 10 120 python3 bench.py --steps 4000 --warmup 200 --no-cpu-baseline > gpurun_out/ab_single.json 2>&1 || exit 1
for f in ab_fork ab_single; do python3 -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f', d['ms_per_step']*1000, 'us')"; done
