# r04: cfg3 ConvLSTM video bench with the SLP-vectorized libptlstm (exp/) vs
# the release (-fno-slp-vectorize) build, then rocprof kernel stats of the release.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=pathtracker-models_amd/ptamd
ARGS="--video --filt 7 --timesteps 64 --no-cpu-baseline --steps 6 --warmup 2"
timeout -k 10 300 python tools/bench_convlstm.py $ARGS > gpurun_out/i_rel.json 2> gpurun_out/i_rel.err
r=$?; echo REL_EXIT $r; cut -c1-300 gpurun_out/i_rel.json; [ $r -eq 0 ] || exit $r
cp $L/libptlstm.so /tmp/rel_lstm.so; cp exp/libptlstm_slp.so $L/libptlstm.so
timeout -k 10 300 python tools/bench_convlstm.py $ARGS > gpurun_out/i_slp.json 2> gpurun_out/i_slp.err
r=$?; echo SLP_EXIT $r; cut -c1-300 gpurun_out/i_slp.json; cp /tmp/rel_lstm.so $L/libptlstm.so; [ $r -eq 0 ] || exit $r
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/i_prof -o lprof -- python3 tools/bench_convlstm.py --video --filt 7 --timesteps 64 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/i_prof.log 2>&1
r=$?; echo PROF_EXIT $r; f=$(find gpurun_out/i_prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-5 "$f" | head -16 | cut -c1-150
exit $r
