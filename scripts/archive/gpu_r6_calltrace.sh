# Round 6: kernel timeline of update_many(20) calls (MNIST) -- where the short call's fixed cost sits
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6ct2
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/scripts/call_trace.py 20 > $GRAFT_REPO_ROOT/$O/call_trace.txt 2>&1 || { tail $GRAFT_REPO_ROOT/$O/call_trace.txt; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/call_gaps2.py $O/kt > $O/gaps.txt || exit 1
cat $O/gaps.txt
