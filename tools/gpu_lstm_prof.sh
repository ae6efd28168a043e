# ConvLSTM cfg3 (video, k=7, 32x32x64f, B=256 bf16): the bench line and a
# rocprofv3 kernel-trace + stats pass of it (TAG names the outputs).
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-l}
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_convlstm.py --video --filt 7 --no-cpu-baseline > gpurun_out/${TAG}_lstm_bench.json 2> gpurun_out/${TAG}_lstm_bench.err
r=$?; echo LSTM_BENCH_EXIT $r; cat gpurun_out/${TAG}_lstm_bench.json; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_lstm_bench.err; exit $r; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_lprof -o run -- python3 tools/bench_convlstm.py --video --filt 7 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_lprof.log 2>&1
r=$?; echo LSTM_PROF_EXIT $r; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_lprof.log; exit $r; }
f=$(ls gpurun_out/${TAG}_lprof/run_kernel_stats.csv gpurun_out/${TAG}_lprof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/${TAG}_lstm_kernel_stats.csv
python3 - gpurun_out/${TAG}_lstm_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:60]:60s} n={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:8.2f}us tot={float(r["TotalDurationNs"])/1e6:8.2f}ms')
PY
exit 0
