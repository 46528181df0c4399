# Round 4, config 5: bf16 parity tests of the step forms, then interleaved 300-step synth
# benches: the default against each arm (ENV=VAL[,ENV2=VAL2] per arm).
# usage: gpu_r4_bf.sh [arm ...]   e.g. VAEB_BF_SPLIT2=1,VAEB_BF_FORK=2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/bf
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_bf16.py \
  -k "${BF_TESTS:-two_slices or split2 or forked}" > gpurun_out/bf/tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/bf/tests.log | head -20; tail -5 gpurun_out/bf/tests.log; exit 1; }
tail -1 gpurun_out/bf/tests.log
for r in 1 2; do
  for arm in base "$@"; do
    envs=""; [ $arm != base ] && envs=$(echo $arm | tr ',' ' ')
    env $envs timeout -k 10 300 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/bf/s.json 2> gpurun_out/bf/s.err || { tail gpurun_out/bf/s.err; exit 1; }
    cp gpurun_out/bf/s.json "gpurun_out/bf/s_${arm}_r$r.json"
    python3 -c "import json;d=json.load(open('gpurun_out/bf/s.json'));print('$arm', round(d['ms_per_step']*1000,1), 'us/step')"
  done
done
