# Diagnostics: MNIST bench with and without an env switch, interleaved rounds: env_ab2.sh VAR=VAL [VAR2=VAL2 ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in $(seq ${AB_ROUNDS:-2}); do
  for v in base "$@"; do
    if [ $v = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/x.json 2> gpurun_out/ab/x.err || { tail -5 gpurun_out/ab/x.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/x.json'));print('$v', round(d['ms_per_step']*1000,2), {k: round(v*1000,2) for k,v in d['kernels_ms'].items()})"
  done
done
