# GPU performance check: plain bench, counter list, one PMC pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > gpurun_out/bench_plain.json 2> gpurun_out/bench_plain.err || exit 1
cat gpurun_out/bench_plain.json
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
grep -o -E "^[[:space:]]*[A-Z][A-Z0-9_]+" gpurun_out/counters_list.txt | sort -u | tr '\n' ' ' | head -c 3000 > gpurun_out/counter_names.txt
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc1 -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/pmc1.json 2> gpurun_out/pmc1.err
echo "pmc rc=$?"
ls gpurun_out/pmc1
