# Round 5: timing-only knock-out builds (wrong results; VAEB_KO_* in kernels_aux.hpp / latent.hpp)
# of the last launch and the decoder, 2000-step bench lines each, then the call-overhead
# variants (VAEB_SYNC_SPIN, VAEB_EAGER_FIRST) in the driver's 20 / 5 form, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ko
mkdir -p $O
for v in ${VARIANTS:-default kw3p kw3x kw3d kw3s kds kdw kde default}; do
  if [ $v = default ]; then L=""; else L=$v; fi
  VAEB_LIB_VARIANT=$L timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/b_$v.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$v.json'));print('$v', round(d['ms_per_step']*1000,2), {k: round(x*1000,2) for k,x in d['kernels_ms'].items()})"
done
for rep in 1 2 3; do
  for cv in "0 1" "1 1" "0 0" "1 0"; do
    set -- $cv
    VAEB_SYNC_SPIN=$1 VAEB_EAGER_FIRST=$2 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/d_$1$2_$rep.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/d_$1$2_$rep.json'));print('spin $1 eager $2', round(d['ms_per_step']*1000,2))"
  done
done
