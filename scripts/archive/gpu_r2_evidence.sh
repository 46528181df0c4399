# Round-2 evidence: rocprof kernel traces + PMC passes per config, MFMA busy, bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_profile_round2.sh || exit 1
# the bench lines below read `traffic` from profiles/r2: use this run's PMC passes
for cfg in mnist frey fv fvs synth; do cp gpurun_out/round2/$cfg/pmc_per_launch.json profiles/r2/pmc_${cfg}_per_launch.json; done
bash scripts/gpu_mfma_busy.sh || exit 1
mkdir -p gpurun_out/lines2
for cfg in mnist frey fv fvs synth; do
  timeout -k 10 300 python3 bench.py --config $cfg > gpurun_out/lines2/$cfg.json 2> gpurun_out/lines2/$cfg.err || { tail gpurun_out/lines2/$cfg.err; exit 1; }
done
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/lines2/driver_form.json 2> gpurun_out/lines2/driver_form.err || exit 1
python3 -c "
import json
for c in ('mnist','frey','fv','fvs','synth','driver_form'):
    d=json.load(open('gpurun_out/lines2/%s.json'%c)); r=d['roofline']
    print(c, round(d['ms_per_step']*1000,2), 'us', round(d['value']), 'img/s', r['kernel'], round(r['frac'],4), 'traffic', r['traffic'], 'cpu', round(d.get('cpu_baseline',{}).get('value',0)))"
