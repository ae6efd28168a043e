# r04: ConvLSTM k_lwgrad2 (column-owned weight gradients): LSTM tests (incl.
# the bitwise A/B tests), then cfg3 bench with PT_LWGRAD2=1 (default) and 0.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_lstm_video.py tests/test_gpu_lstm.py > gpurun_out/s_tests.log 2>&1
r=$?; tail -3 gpurun_out/s_tests.log; [ $r -eq 0 ] || { grep -E "assert|Error|FAILED" gpurun_out/s_tests.log | head -20; exit $r; }
for v in 1 0; do
  PT_LWGRAD2=$v timeout -k 10 400 python tools/bench_convlstm.py --video --filt 7 --timesteps 64 > gpurun_out/s_lstm_$v.json 2> gpurun_out/s_lstm_$v.err
  r=$?; echo "LWGRAD2=$v exit $r"; cut -c1-300 gpurun_out/s_lstm_$v.json; [ $r -eq 0 ] || { tail -5 gpurun_out/s_lstm_$v.err; exit $r; }
done
