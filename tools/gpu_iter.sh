# iteration loop on the GPU box (libraries prebuilt in-tree): -m gpu parity,
# per-kernel launch times (tools/ablate.py, MASKS), headline bench; stops at the first failure
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -q -m gpu -p no:cacheprovider -x --timeout 120 --timeout-method thread ${PYARGS} > gpurun_out/i_parity.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -3 gpurun_out/i_parity.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/i_parity.log | head -20; exit $r; }
MASKS=${MASKS:-0} timeout -k 10 300 python tools/ablate.py > gpurun_out/i_ablate.log 2>&1
r=$?; echo ABL_EXIT $r; cat gpurun_out/i_ablate.log | grep -v amdgpu.ids; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/i_bench.json 2> gpurun_out/i_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/i_bench.json; [ $r -eq 0 ] || { tail -5 gpurun_out/i_bench.err; exit $r; }
