# Round 2: long-run A/B of the decout tile shape (VAEB_DECOUT_2B) at config 5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/decout
for r in 1 2 3; do
for v in 0 1; do
  VAEB_DECOUT_2B=$v timeout -k 10 200 python3 bench.py --config synth --steps 3000 --warmup 50 --no-cpu-baseline > gpurun_out/decout/d$v.json 2> gpurun_out/decout/d$v.err || { tail -5 gpurun_out/decout/d$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/decout/d$v.json'));k=d['kernels_ms'];print('2b=$v', round(d['ms_per_step']*1000,1), 'us  decout', round(k['bf_decout']*1000,1), 'dhd', round(k['bf_dhd_dW26']*1000,1))"
done
done
