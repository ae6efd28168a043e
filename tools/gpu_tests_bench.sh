# -m gpu suite (per-test timeout) then the default bench line.  Stops at the
# first failure.  SEL narrows the tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest ${SEL:-tests} -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -rf > gpurun_out/r03_gpu_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -8 gpurun_out/r03_gpu_tests.log; [ $r -eq 0 ] || exit $r
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/r03_bench_tb.json 2> gpurun_out/r03_bench_tb.err
r=$?; echo BENCH_EXIT $r; cut -c1-400 gpurun_out/r03_bench_tb.json; [ $r -eq 0 ] || tail -5 gpurun_out/r03_bench_tb.err
exit $r
