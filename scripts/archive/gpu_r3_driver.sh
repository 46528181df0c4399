# The driver's bench form (--steps 20 --warmup 5, fresh process each) alternated across
# settings: Usage: bash scripts/gpu_r3_driver.sh "VAR=a" "VAR=b" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/driver_ab.txt
for rep in 1 2 3 4; do
  for setting in "$@"; do
    env $setting timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 ${DRV_ARGS} > gpurun_out/drv_line.json 2> gpurun_out/drv.err || { tail -20 gpurun_out/drv.err; exit 1; }
    python3 -c "
import json,sys
d=json.load(open('gpurun_out/drv_line.json')); print(sys.argv[1], round(d['ms_per_step']*1000,2), 'us/step')" "$setting" | tee -a gpurun_out/driver_ab.txt
  done
done
