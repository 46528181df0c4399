# Round 5: kernel traces of the fp32 data-parallel step at world 1, bucket A
# forked onto the second stream (VAEB_DP_OVERLAP=1) and not (=0), and the fused step without a
# communicator, for attributing the fork / join cost (scripts/dp_fork_anatomy.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5dp
mkdir -p $O
for ov in 1 0 none; do
  if [ $ov = none ]; then
    VAEB_DP_NOCOMM=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/ov_$ov -o run -- python3 scripts/dp_fork_probe.py > $O/probe_$ov.txt 2>&1 || { tail $O/probe_$ov.txt; exit 1; }
  else
    VAEB_DP_OVERLAP=$ov timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/ov_$ov -o run -- python3 scripts/dp_fork_probe.py > $O/probe_$ov.txt 2>&1 || { tail $O/probe_$ov.txt; exit 1; }
  fi
  grep "us/step" $O/probe_$ov.txt
  python3 scripts/dp_fork_anatomy.py $O/ov_$ov/run_kernel_trace.csv > $O/anatomy_$ov.txt || exit 1
  head -40 $O/anatomy_$ov.txt
done
