# Autoencoder engine parity tests (degenerate-vae ae.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ae.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ae_tests.log 2>&1; rc=$?
tail -16 gpurun_out/ae_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/ae_tests.log | head -20; exit 1; }
exit 0
