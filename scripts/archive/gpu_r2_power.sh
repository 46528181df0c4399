# Round 2: power / clock while config 5 steps (is the bf16 chain power-capped?).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/power
rocm-smi --showpower --showclocks --showmaxpower > gpurun_out/power/idle.txt 2>&1 || true
( for i in $(seq 1 80); do date +%s.%N; rocm-smi --showpower --showclocks 2>&1 | grep -E "Power|sclk|fclk|mclk"; sleep 0.2; done ) > gpurun_out/power/samples.txt 2>&1 &
SAMP=$!
timeout -k 10 200 python3 bench.py --config synth --steps 20000 --warmup 20 --no-cpu-baseline > gpurun_out/power/b.json 2> gpurun_out/power/b.err || { tail -5 gpurun_out/power/b.err; kill $SAMP; exit 1; }
wait $SAMP
python3 -c "import json;d=json.load(open('gpurun_out/power/b.json'));print(round(d['ms_per_step']*1000,1))"
grep -iE "max|power" gpurun_out/power/idle.txt | head
grep -E "Power" gpurun_out/power/samples.txt | sort | uniq -c | sort -rn | head -8
grep -E "sclk" gpurun_out/power/samples.txt | sort | uniq -c | sort -rn | head -8
