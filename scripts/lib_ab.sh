# Diagnostics: MNIST bench for the default library and in-tree variants
# (vaeb_amd/libvaeb_hip_<v>.so, VAEB_LIB_VARIANT=<v>), interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in $(seq ${AB_ROUNDS:-2}); do
  for v in base "$@"; do
    if [ $v = base ]; then unset VAEB_LIB_VARIANT; else export VAEB_LIB_VARIANT=$v; fi
    timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || { tail -5 gpurun_out/ab/$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));print('$v', round(d['ms_per_step']*1000,2), {k: round(v*1000,2) for k,v in d['kernels_ms'].items()})"
  done
done
