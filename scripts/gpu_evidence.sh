# Round evidence for every bench config, in one call: kernel-trace stats, FETCH_SIZE and
# WRITE_SIZE PMC passes (separate runs, MI355X_MICROARCH.md §HBM), the MFMA-busy pass, then
# the bench line with the CPU baseline (it reads the PMC traffic just copied into profiles/${ROUND:-r3}).
# -> gpurun_out/round/<config>/ and profiles/${ROUND:-r3}/ (the box's copy; merged back via gpurun_out)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT/profiles profiles/${ROUND:-r3}
for cfg in ${CONFIGS:-mnist frey fv fvs synth}; do
  O=$OUT/$cfg
  mkdir -p $O
  if [ $cfg = synth ]; then S="--steps 30 --warmup 3"; P="--steps 10 --warmup 2"; else S="--steps 1000 --warmup 100"; P="--steps 200 --warmup 20"; fi
  pre="${cfg}_"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config $cfg $S --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err || { tail $O/bench_trace.err; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --config $cfg $P --no-cpu-baseline > /dev/null 2> $O/fetch.err || { tail $O/fetch.err; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --config $cfg $P --no-cpu-baseline > /dev/null 2> $O/write.err || { tail $O/write.err; exit 1; }
  python3 scripts/pmc_summary.py $O/pmc_per_launch.json $O/fetch $O/write > $O/pmc_summary.txt || exit 1
  if [ $cfg != fv ] && [ $cfg != fvs ]; then
    timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o run -- python3 bench.py --config $cfg $P --no-cpu-baseline > /dev/null 2> $O/mfma.err || { tail $O/mfma.err; exit 1; }
    python3 scripts/pmc_summary.py $O/pmc_mfma.json $O/mfma > /dev/null || exit 1
    python3 scripts/mfma_busy.py $cfg $O/pmc_mfma.json > $O/mfma_busy.txt || exit 1
    cp $O/mfma_busy.txt $OUT/profiles/mfma_busy_$cfg.txt
    cp $O/pmc_mfma.json $OUT/profiles/pmc_mfma_${cfg}_per_launch.json
  fi
  cp $O/trace/run_kernel_stats.csv $OUT/profiles/${pre}kernel_stats.csv
  cp $O/pmc_summary.txt $OUT/profiles/${pre}pmc_summary.txt
  cp $O/pmc_per_launch.json $OUT/profiles/pmc_${cfg}_per_launch.json
  cp $O/pmc_per_launch.json profiles/${ROUND:-r3}/pmc_${cfg}_per_launch.json
  [ $cfg = mnist ] && cp $O/trace/run_domain_stats.csv $OUT/profiles/domain_stats.csv
  timeout -k 10 300 python3 bench.py --config $cfg > $O/bench_line.json 2> $O/bench_line.err || { tail $O/bench_line.err; exit 1; }
  cp $O/bench_line.json $OUT/profiles/${pre}bench_line.json
  echo "== $cfg"; cut -c1-150 $O/trace/run_kernel_stats.csv | head -8
  python3 -c "
import json; d=json.load(open('$O/bench_line.json'))
r=d['roofline']; c=d.get('cpu_baseline',{})
print('$cfg', round(d['value']), d['unit'], 'us/step', round(d['ms_per_step']*1000,2), 'roofline', r['kernel'], round(r['frac'],4), 'traffic', r['traffic'], 'cpu', round(c.get('value',0)), c.get('cores'))"
done
