# r04: XCD-affine workgroup order: GPU tests on it, then per-launch times
# with PT_XCD_MAP=0 / 1 interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider -x --timeout 150 --timeout-method thread > gpurun_out/g_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/g_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/g_tests.log | head -30; exit $r; }
MASKS="0:PT_XCD_MAP=0,0:PT_XCD_MAP=1" ROUNDS=3 timeout -k 10 300 python -u tools/ablate.py > gpurun_out/g_ablate.log 2>&1
r=$?; echo ABLATE_EXIT $r; grep -v amdgpu.ids gpurun_out/g_ablate.log | tail -5
exit $r
