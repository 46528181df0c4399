# Round 6 A/B: the 16-bit step's bias optimizer + ELBO on a third stream right after dh (beside dW3)
# buffered) instead of at the step's end (VAEB_LIB_VARIANT=base: the build before)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6s4
mkdir -p $O
true
true
for r in 1 2 3 4; do
  for v in base new; do
    if [ $v = base ]; then export VAEB_LIB_VARIANT=base; else unset VAEB_LIB_VARIANT; fi
    timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > $O/s_${v}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/s_${v}_$r.json'));print('$v $r', round(d['ms_per_step']*1000,1))"
  done
done
