# Round 6 A/B: slab-form encoder with 2 vs 4 h column tiles per workgroup (VAEB_ENC_CT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6ct
mkdir -p $O
us() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['ms_per_step']*1000,2), 'us/step')"; }
VAEB_ENC_CT=4 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_step.py -x -q --timeout 120 --timeout-method thread \
  -k "atomic_and_slab or deferred_dw2 or mnist" > $O/tests_ct4.txt 2>&1 || { tail -30 $O/tests_ct4.txt; exit 1; }
tail -2 $O/tests_ct4.txt
for r in 1 2; do
  for ct in 2 4; do
    VAEB_ENC_CT=$ct timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_${ct}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    us $O/driver_${ct}_$r.json "driver ct$ct $r"
    VAEB_ENC_CT=$ct timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/m2000_${ct}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    us $O/m2000_${ct}_$r.json "2000 ct$ct $r"
  done
done
cd /tmp
for ct in 2 4; do
  VAEB_ENC_CT=$ct timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof$ct -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 500 --warmup 50 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_$ct.log 2>&1 || exit 1
done
