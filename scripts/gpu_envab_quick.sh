# Diagnostics: bench with one env var swept (no tests), interleaved rounds.
# Usage: gpu_envab_quick.sh VAR "v1 v2" [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VAR=$1; VALS=$2; shift 2
mkdir -p gpurun_out/envab
for r in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline "$@" > gpurun_out/envab/v$v.json 2> gpurun_out/envab/v$v.err || { tail -5 gpurun_out/envab/v$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/envab/v$v.json'));print('$VAR=$v', round(d['ms_per_step']*1000,2), 'us', {k: round(x*1000,2) for k,x in d['kernels_ms'].items()}, 'elbo', round(d['elbo'],4))"
  done
done
