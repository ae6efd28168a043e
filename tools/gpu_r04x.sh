# r04: ConvLSTM transposed conv on 8 waves (PT_LCONVT8): LSTM tests, then cfg3
# bench with PT_LCONVT8=1 (default) and 0.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_lstm_video.py tests/test_gpu_lstm.py > gpurun_out/x_tests.log 2>&1
r=$?; tail -3 gpurun_out/x_tests.log; [ $r -eq 0 ] || { grep -E "assert|Error|FAILED" gpurun_out/x_tests.log | head -20; exit $r; }
for v in 1 0; do
  PT_LCONVT8=$v timeout -k 10 400 python tools/bench_convlstm.py --video --filt 7 --timesteps 64 > gpurun_out/x_lstm_$v.json 2> gpurun_out/x_lstm_$v.err
  r=$?; echo "LCONVT8=$v exit $r"; cut -c1-300 gpurun_out/x_lstm_$v.json; [ $r -eq 0 ] || { tail -5 gpurun_out/x_lstm_$v.err; exit $r; }
done
