# GPU check: parity tests (per-test timeout), smoke, short bench. Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -v -m gpu -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/c_parity.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -4 gpurun_out/c_parity.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/c_parity.log | head -30; exit $r; }
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/c_smoke.log 2>&1
r=$?; echo SMOKE_EXIT $r; tail -3 gpurun_out/c_smoke.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/c_bench.json 2> gpurun_out/c_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/c_bench.json; [ $r -eq 0 ] || tail -8 gpurun_out/c_bench.err
exit $r
