# r06 first GPU pass: the fused / trace GPU tests on the rebuilt libraries,
# the HW_ID phase trace (tools/trace.py), the A/B of the PT_EI_FULL and
# persistent-forward builds (tools/libab.py) and the PT_EI_FULL accuracy
# drift (tools/ei_drift.py).  Stops at the first failing step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_trace.py tests/test_gpu_dist.py tests/test_gpu_lstm_video.py -v -m gpu -p no:cacheprovider -x --timeout 200 --timeout-method thread > gpurun_out/r06a_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -3 gpurun_out/r06a_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r06a_tests.log | head -30; exit $r; }
TAG=r06a timeout -k 10 200 python -u tools/trace.py > gpurun_out/r06a_trace.txt 2>&1
r=$?; echo TRACE_EXIT $r; [ $r -eq 0 ] || { tail -20 gpurun_out/r06a_trace.txt; exit $r; }
ROUNDS=${ROUNDS:-5} timeout -k 10 400 python -u tools/libab.py > gpurun_out/r06a_libab.txt 2>&1
r=$?; echo LIBAB_EXIT $r; cat gpurun_out/r06a_libab.txt | grep -v amdgpu.ids; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u tools/ei_drift.py > gpurun_out/r06a_ei_drift.txt 2>&1
r=$?; echo DRIFT_EXIT $r; tail -5 gpurun_out/r06a_ei_drift.txt; exit $r
