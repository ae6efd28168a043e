# GPU parity (whole -m gpu suite) + headline bench + cfg4 hGRU bench; stops at the first failure.
# Libraries are prebuilt in-tree on the CPU side.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -q -m gpu -p no:cacheprovider -x --timeout 120 --timeout-method thread ${PYARGS} > gpurun_out/t_parity.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -3 gpurun_out/t_parity.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_parity.log | head -20; exit $r; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/t_bench.json 2> gpurun_out/t_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/t_bench.json; [ $r -eq 0 ] || { tail -5 gpurun_out/t_bench.err; exit $r; }
timeout -k 10 400 python tools/bench_hgru.py ${HGARGS} > gpurun_out/t_hgru.json 2> gpurun_out/t_hgru.err
r=$?; echo HGRU_EXIT $r; cat gpurun_out/t_hgru.json; [ $r -eq 0 ] || { tail -5 gpurun_out/t_hgru.err; exit $r; }
