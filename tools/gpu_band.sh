# Banded backward conv: bitwise tests, then timing A/B.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -rf -k band > gpurun_out/band_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -5 gpurun_out/band_tests.log; [ $r -eq 0 ] || exit $r
MASKS="0:PT_CONV_BAND=0,0:PT_CONV_BAND=1" ROUNDS=3 timeout -k 10 200 python tools/ablate.py > gpurun_out/abl_band.log 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/abl_band.log | tail -4; exit $r
