# r04: ConvLSTM conversions / column sums: the LSTM GPU tests, then the cfg3 bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_lstm_video.py -v -m gpu -p no:cacheprovider -x --timeout 150 --timeout-method thread > gpurun_out/j_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/j_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/j_tests.log | head -30; exit $r; }
timeout -k 10 400 python tools/bench_convlstm.py --video --filt 7 --timesteps 64 > gpurun_out/j_lstm.json 2> gpurun_out/j_lstm.err
r=$?; echo LSTM_EXIT $r; cut -c1-900 gpurun_out/j_lstm.json; [ $r -eq 0 ] || tail -5 gpurun_out/j_lstm.err
exit $r
