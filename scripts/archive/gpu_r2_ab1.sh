# Round 2: the driver's bench command after the graph-family fix, then base vs the fenced
# slab hand-off (VAEB_SLAB_ACQREL) with a parity check of the variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_driver.json'));print('driver-form 20/5', round(d['ms_per_step']*1000,2), 'us')"
done
VAEB_LIB_VARIANT=acqrel timeout -k 10 300 python3 -u -m pytest tests/test_gpu_step.py -q --timeout 120 --timeout-method thread -m gpu -k "mnist20 or frey2 or trajectory or B1024" > gpurun_out/acqrel_tests.log 2>&1 || { tail -30 gpurun_out/acqrel_tests.log; exit 1; }
tail -2 gpurun_out/acqrel_tests.log
bash scripts/lib_ab.sh acqrel
