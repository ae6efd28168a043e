# r04: ConvLSTM with 2-row weight-gradient bands as the default: LSTM tests,
# then the cfg3 bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_lstm_video.py tests/test_gpu_lstm.py > gpurun_out/u_tests.log 2>&1
r=$?; tail -2 gpurun_out/u_tests.log; [ $r -eq 0 ] || { grep -E "assert|Error|FAILED" gpurun_out/u_tests.log | head -20; exit $r; }
timeout -k 10 400 python tools/bench_convlstm.py --video --filt 7 --timesteps 64 > gpurun_out/u_lstm.json 2> gpurun_out/u_lstm.err
r=$?; echo "bench exit $r"; cut -c1-300 gpurun_out/u_lstm.json; exit $r
