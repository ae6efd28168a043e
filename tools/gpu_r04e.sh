# r04: k_pw_bb2 correctness (A/B vs k_pw_bb, reference goldens, headline
# parity) then per-launch times of both (interleaved in one process).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_pwb2.py tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider -x --timeout 150 --timeout-method thread > gpurun_out/e_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/e_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/e_tests.log | head -30; exit $r; }
MASKS="0:PT_PWB2=0+PT_PWA2=0,0:PT_PWB2=1+PT_PWA2=1" ROUNDS=3 timeout -k 10 300 python -u tools/ablate.py > gpurun_out/e_ablate.log 2>&1
r=$?; echo ABLATE_EXIT $r; grep -v amdgpu.ids gpurun_out/e_ablate.log | tail -8
exit $r
