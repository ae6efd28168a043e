# ConvLSTM bench + rocprofv3 kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$NOBENCH" ] || timeout -k 10 300 python tools/bench_convlstm.py ${ARGS} > gpurun_out/lb.json 2> gpurun_out/lb.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/lb.json; [ $r -eq 0 ] || { tail -5 gpurun_out/lb.err; exit $r; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof -o lprof -- python tools/bench_convlstm.py --steps 3 --warmup 1 --no-cpu-baseline ${ARGS} > gpurun_out/lprof.log 2>&1
r=$?; echo PROF_EXIT $r; find gpurun_out/lprof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/lprof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-5 "$f" | head -25 | cut -c1-160
exit $r
