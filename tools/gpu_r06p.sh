# r06: band2's fill prefetch (PT_FILL_PRE) -- bitwise tests, then the A/B
# against ptamd/ab/libptcell_nopre.so.  Every GPU step under its own limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -k "band or split_pair or tiled" -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06p_tests.log 2>&1
r=$?; tail -4 gpurun_out/r06p_tests.log; [ $r -eq 0 ] || exit $r
ROUNDS=5 timeout -k 10 300 python -u tools/libab.py > gpurun_out/r06p_libab.txt 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/r06p_libab.txt; exit $r
