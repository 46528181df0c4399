# HIP runtime knobs vs the MNIST step (graph replays): one bench line per setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/env
run() {
    name=$1; shift
    env "$@" timeout -k 10 120 python3 bench.py --steps 4000 --warmup 500 --no-cpu-baseline > gpurun_out/env/$name.json 2> gpurun_out/env/$name.err || return 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/env/$name.json')); print('$name', round(d['ms_per_step']*1000,2), 'us/step')"
}
run base A=1 &&
run devkarg1 HIP_FORCE_DEV_KERNARG=1 &&
run devkarg0 HIP_FORCE_DEV_KERNARG=0 &&
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 &&
run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 &&
run base2 A=1
