# Short measurement on the GPU box (TAG names the outputs): the bench line
# (no CPU baseline, no f32 figure) and a rocprofv3 kernel-trace + stats pass
# of the same command; every GPU step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-m}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-f32 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/${TAG}_bench.json; [ $r -eq 0 ] || { tail -8 gpurun_out/${TAG}_bench.err; exit $r; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32 ${BENCH_ARGS:-} > gpurun_out/${TAG}_prof.log 2>&1
r=$?; echo PROF_EXIT $r; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_prof.log; exit $r; }
f=$(ls gpurun_out/${TAG}_prof/run_kernel_stats.csv gpurun_out/${TAG}_prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/${TAG}_kernel_stats.csv
python3 - gpurun_out/${TAG}_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:60]:60s} n={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:8.2f}us tot={float(r["TotalDurationNs"])/1e6:8.2f}ms')
PY
exit 0
