# Round 4 evidence lines: the driver's short form (K = 20, W = 5) three times, a 2000-step MNIST
# line, a 300-step config-5 line, and the default-form stage stamps (timeline build).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lines
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_form_$i.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/driver_form_$i.json'));print('driver form', round(d['ms_per_step']*1000,2))"
done
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline > $O/mnist_2000.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "import json;d=json.load(open('$O/mnist_2000.json'));print('mnist 2000', round(d['ms_per_step']*1000,2))"
timeout -k 10 300 python3 bench.py --config synth --steps 300 --warmup 20 --no-cpu-baseline > $O/synth_300.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "import json;d=json.load(open('$O/synth_300.json'));print('synth 300', round(d['ms_per_step']*1000,1))"
timeout -k 10 120 python3 scripts/tl_dump.py mnist > /dev/null && timeout -k 10 120 python3 scripts/tl_stages.py > $O/tl_stages.txt 2>&1 || exit 1
cp gpurun_out/tl_mnist.npz $O/ 2>/dev/null || true
