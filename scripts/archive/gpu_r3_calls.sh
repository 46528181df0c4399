# Round 3: per-call fixed cost A/B, host-ELBO / eager-sync correctness, DP fork trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/call_ab.py > gpurun_out/call_ab.txt 2>&1 || { tail -20 gpurun_out/call_ab.txt; exit 1; }
cat gpurun_out/call_ab.txt
VAEB_ELBO_HOST=1 VAEB_SYNC_EAGER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_hostelbo.log 2>&1 || { tail -30 gpurun_out/tests_hostelbo.log; exit 1; }
tail -2 gpurun_out/tests_hostelbo.log
for ov in 1 0; do
  VAEB_DP_OVERLAP=$ov timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dpfork$ov -o dpfork -- python3 scripts/dp_fork_probe.py > gpurun_out/dpfork$ov.txt 2>&1 || { tail -20 gpurun_out/dpfork$ov.txt; exit 1; }
  grep "us/step" gpurun_out/dpfork$ov.txt
  f=$(find gpurun_out/dpfork$ov -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_gaps.py "$f" 320 > gpurun_out/dpfork${ov}_gaps.txt && cat gpurun_out/dpfork${ov}_gaps.txt
done
