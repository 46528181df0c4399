# bf16 engine: split-K slices of heads (h [W4|W5]) and dz (dA1 W1^T): default (4 / 8) vs
# fewer slices (interleaved config-5 runs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ks
for r in 1 2; do
for v in "4 8" "2 8" "4 4" "2 4" "2 2"; do
  set -- $v
  VAEB_BF_KS_HEADS=$1 VAEB_BF_KS_DZ=$2 timeout -k 10 200 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/ks/s.json 2> gpurun_out/ks/s.err || { tail -5 gpurun_out/ks/s.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ks/s.json'));k=d['kernels_ms'];print('heads=$1 dz=$2', round(d['ms_per_step']*1000,1), 'us', d['elbo'], {x: round(k[x]*1000,1) for x in ('bf_heads','bf_latent','bf_dz','bf_latent_bwd')})"
done
done
