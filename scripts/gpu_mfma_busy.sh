# MFMA-busy evidence per config (north star: "rocprof HBM GB/s and MFMA-busy counters
# against chip peak"): one --pmc pass per config with the SQ MFMA counters and the GRBM
# clock, folded per launch by scripts/pmc_summary.py, then scripts/mfma_busy.py.
# -> gpurun_out/mfma/<config>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in mnist frey synth; do
  O=gpurun_out/mfma2/$cfg
  mkdir -p $O
  if [ $cfg = synth ]; then P="--steps 10 --warmup 2"; else P="--steps 200 --warmup 20"; fi
  timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 bench.py --config $cfg $P --no-cpu-baseline > /dev/null 2> $O/p1.err || { tail $O/p1.err; exit 1; }
  python3 scripts/pmc_summary.py $O/pmc_per_launch.json $O/p1 > /dev/null || exit 1
  python3 scripts/mfma_busy.py $cfg $O/pmc_per_launch.json > $O/mfma_busy.txt || exit 1
  cat $O/mfma_busy.txt
done
