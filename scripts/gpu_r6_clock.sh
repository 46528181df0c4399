# Round 6: config 5, fp16 vs bf16 operands -- per-kernel cycles over duration (the clock the chip
# held), to test whether the fp16 instantiation's faster epilogue launches are a clock effect
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6clk
mkdir -p $O
for dt in fp16 bf16; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/$dt -o run -- python3 bench.py --config synth --dtype $dt --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2> $O/$dt.err || { tail $O/$dt.err; exit 1; }
  echo "== $dt"
  python3 scripts/clock_per_kernel.py $O/$dt | head -12 || exit 1
done
