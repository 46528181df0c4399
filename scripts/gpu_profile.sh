# Round profile: kernel trace + stats, and the HBM-traffic PMC passes (FETCH_SIZE and
# WRITE_SIZE in separate passes, per MI355X_MICROARCH.md), on a short bench run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1/trace -o run -- python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/prof_r1/bench_trace.json 2> gpurun_out/prof_r1/bench_trace.err || exit 1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_r1/fetch -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r1/bench_fetch.json 2> gpurun_out/prof_r1/bench_fetch.err || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_r1/write -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r1/bench_write.json 2> gpurun_out/prof_r1/bench_write.err || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof_r1/insts -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r1/bench_insts.json 2> gpurun_out/prof_r1/bench_insts.err
echo "rc=$?"
ls -R gpurun_out/prof_r1 | head -30
