# GPU tests + smoke on the GPU box (TAG names the outputs under gpurun_out/);
# PYTEST_ARGS narrows the selection (default: the whole -m gpu suite).  Stops at
# the first failure; every GPU step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-t}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${PYTEST_ARGS:-tests} -v -m gpu -p no:cacheprovider -x --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/${TAG}_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_tests.log | head -30; exit $r; }
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1
r=$?; echo SMOKE_EXIT $r; tail -1 gpurun_out/${TAG}_smoke.log
cp gpurun_out/parity_records.json gpurun_out/${TAG}_parity_records.json 2>/dev/null
exit $r
