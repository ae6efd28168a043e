# r06: the fused forward on tiled frames (xb_exchange) -- bitwise tests, then
# the cfg4 A/B against the split tiled forward (ptamd/ab/libptcell_splitfwd.so)
# and the cfg4 bench.  Every GPU step under its own time limit; stop at the
# first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -k "tiled" -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06t_tests.log 2>&1
r=$?; tail -15 gpurun_out/r06t_tests.log; [ $r -eq 0 ] || exit $r
CELL=hgru HW=64 B=128 T=128 ROUNDS=3 timeout -k 10 300 python -u tools/libab.py > gpurun_out/r06t_libab.txt 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/r06t_libab.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u tools/bench_hgru.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06t_hgru_bench.txt 2>&1
r=$?; tail -3 gpurun_out/r06t_hgru_bench.txt; exit $r
