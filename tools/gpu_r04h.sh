# r04: secondary configs at HEAD: hGRU 64x64x128 (cfg4) and the clip
# ConvLSTM (cfg3, --video --filt 7), one bench line each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/bench_hgru.py --cpu-seconds 10 > gpurun_out/h_hgru.json 2> gpurun_out/h_hgru.err
r=$?; echo HGRU_EXIT $r; cat gpurun_out/h_hgru.json | cut -c1-600; [ $r -eq 0 ] || { tail -5 gpurun_out/h_hgru.err; exit $r; }
timeout -k 10 400 python tools/bench_convlstm.py --video --filt 7 --timesteps 64 > gpurun_out/h_lstm.json 2> gpurun_out/h_lstm.err
r=$?; echo LSTM_EXIT $r; cat gpurun_out/h_lstm.json | cut -c1-600; [ $r -eq 0 ] || tail -5 gpurun_out/h_lstm.err
exit $r
