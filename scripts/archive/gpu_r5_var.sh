# Round 5: 2000-step bench lines for a list of "variant:ENV=VAL" entries (variant = in-tree
# libvaeb_hip_<variant>.so or "default"), in order.  Usage: RUNS="base:X=1 base:X=0" bash scripts/gpu_r5_var.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5var
mkdir -p $O
i=0
for r in $RUNS; do
  v=${r%%:*}; e=${r#*:}; [ "$e" = "$r" ] && e=""; e=${e//,/ }
  if [ $v = default ]; then L=""; else L=$v; fi
  i=$((i+1))
  env VAEB_LIB_VARIANT=$L $e timeout -k 10 200 python3 bench.py --steps ${STEPS:-2000} --warmup ${WARM:-200} --no-cpu-baseline $BARGS > $O/b_$i.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$i.json'));print('$r', round(d['ms_per_step']*1000,2), {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
done
