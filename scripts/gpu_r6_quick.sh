# Round 6: quick lines on the current build -- MNIST driver form (20 / 5) x3, MNIST 2000 steps,
# config 5 with bf16 and fp16 operands (300 steps, alternating) -> gpurun_out/r6q/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6q
mkdir -p $O
us() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['ms_per_step']*1000,2), 'us/step', d.get('dtype'))"; }
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_$i.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  us $O/driver_$i.json "driver form $i"
done
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/mnist_2000.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
us $O/mnist_2000.json "mnist 2000"
for r in 1 2; do
  for dt in bf16 fp16; do
    timeout -k 10 300 python3 bench.py --config synth --dtype $dt --steps 300 --warmup 20 --no-cpu-baseline > $O/synth_${dt}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    us $O/synth_${dt}_$r.json "synth $dt $r"
  done
done
