# r04: full GPU suite + smoke at HEAD (after the ConvLSTM changes).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider -x --timeout 150 --timeout-method thread > gpurun_out/y_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/y_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/y_tests.log | head -20; exit $r; }
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/y_smoke.log 2>&1
r=$?; echo SMOKE_EXIT $r; tail -1 gpurun_out/y_smoke.log; exit $r
