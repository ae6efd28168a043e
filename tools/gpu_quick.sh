# quick GPU iteration: parity tests, kernel timings, bench (stops at the first failure)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
python __graft_entry__.py build > gpurun_out/q_build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/q_build.log; exit 1; }
timeout -k 10 400 python -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/q_parity.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -3 gpurun_out/q_parity.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/q_parity.log | head -20; exit $r; }
MASKS=${MASKS:-0,1} timeout -k 10 300 python tools/ablate.py > gpurun_out/q_ablate.log 2>&1
r=$?; echo ABL_EXIT $r; cat gpurun_out/q_ablate.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/q_bench.json; [ $r -eq 0 ] || tail -5 gpurun_out/q_bench.err
