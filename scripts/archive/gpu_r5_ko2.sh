# Round 5: knock-out variants, 2000-step bench lines, alternating with the default (VARIANTS list).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ko2
mkdir -p $O
for v in ${VARIANTS:-default kaw kah kad kam default}; do
  if [ $v = default ]; then L=""; else L=$v; fi
  VAEB_LIB_VARIANT=$L timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline $BARGS > $O/b_$v.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$v.json'));print('$v', round(d['ms_per_step']*1000,2), {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
done
