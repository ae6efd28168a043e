# r04: ConvLSTM weight gradients with 2-row bands (exp/libptlstm_lwrb2.so, two
# workgroups per CU) against 4-row bands: cfg3 bench each, LSTM video tests
# on the variant first.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=pathtracker-models_amd/ptamd/libptlstm.so
cp $L /tmp/libptlstm_base.so
timeout -k 10 300 python tools/bench_convlstm.py --video --filt 7 --timesteps 64 > gpurun_out/t_base.json 2> gpurun_out/t_base.err
r=$?; echo "base exit $r"; cut -c1-260 gpurun_out/t_base.json; [ $r -eq 0 ] || exit $r
cp exp/libptlstm_lwrb2.so $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_lstm_video.py > gpurun_out/t_tests.log 2>&1
r=$?; tail -2 gpurun_out/t_tests.log; [ $r -eq 0 ] || { cp /tmp/libptlstm_base.so $L; exit $r; }
timeout -k 10 300 python tools/bench_convlstm.py --video --filt 7 --timesteps 64 > gpurun_out/t_lwrb2.json 2> gpurun_out/t_lwrb2.err
r=$?; echo "lwrb2 exit $r"; cut -c1-260 gpurun_out/t_lwrb2.json
cp /tmp/libptlstm_base.so $L
exit $r
