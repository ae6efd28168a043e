# A/B iteration on the GPU box (libraries prebuilt in-tree): parity of a forced
# kernel variant (VARENV, e.g. PT_CELL_BB_RPP=8) on the oracle-pinned tests,
# interleaved per-launch timings of the variants (MASKS, tools/ablate.py), the
# headline bench line.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v}
env ${VARENV} timeout -k 10 400 python -u -m pytest ${PYTESTS:-tests/test_gpu_parity.py tests/test_gpu_edges.py} -q -m gpu -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_parity.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -3 gpurun_out/${TAG}_parity.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_parity.log | head -20; exit $r; }
timeout -k 10 300 python tools/ablate.py > gpurun_out/${TAG}_ablate.log 2>&1
r=$?; echo ABL_EXIT $r; grep -v amdgpu.ids gpurun_out/${TAG}_ablate.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/${TAG}_bench.json; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $r; }
