# The three bench lines (with the CPU baseline leg) -> gpurun_out/lines/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lines
for cfg in mnist frey fv synth; do
  timeout -k 10 300 python3 bench.py --config $cfg > gpurun_out/lines/$cfg.json 2> gpurun_out/lines/$cfg.err || { tail gpurun_out/lines/$cfg.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/lines/$cfg.json'))
r=d['roofline']; c=d.get('cpu_baseline',{})
print('$cfg', round(d['value']), d['unit'], 'ms/step', round(d['ms_per_step'],4), 'roofline', r['kernel'], round(r['frac'],4), 'traffic', r['traffic'], 'cpu', round(c.get('value',0)), c.get('cores'))"
done
