# ConvLSTM GPU parity only
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_lstm.py} -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/l_parity.log 2>&1
r=$?; echo PYTEST_EXIT $r; grep -E "PASSED|FAILED|Error" gpurun_out/l_parity.log | head -40
exit $r
