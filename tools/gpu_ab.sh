# A/B iteration on the GPU box: selected GPU tests (SEL, default the fused
# forward file), then tools/ablate.py over MASKS (interleaved variants in one
# process).  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 400 python -u -m pytest ${SEL:-tests/test_gpu_fused.py} -q -m gpu -p no:cacheprovider -x \
  --timeout 150 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; [ "${SKIP_TESTS:-0}" = 1 ] || tail -3 gpurun_out/ab_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/ab_tests.log | head -20; exit $r; }
MASKS=${MASKS:-0,1} ROUNDS=${ROUNDS:-3} timeout -k 10 300 python tools/ablate.py > gpurun_out/ab_ablate.log 2>&1
r=$?; echo ABL_EXIT $r; grep -v amdgpu.ids gpurun_out/ab_ablate.log; [ $r -eq 0 ] || exit $r
