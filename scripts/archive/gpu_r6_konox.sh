set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/konox
mkdir -p $O
for r in 1 2; do
  for v in base konox; do
    if [ $v = base ]; then unset VAEB_LIB_VARIANT; else export VAEB_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --config synth --steps 100 --warmup 10 --no-cpu-baseline > $O/s_${v}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/s_${v}_$r.json'));print('$v $r', round(d['ms_per_step']*1000,1), {k: round(v*1000,1) for k, v in d.get('kernels_ms', {}).items() if 'dec' in k})"
  done
done
