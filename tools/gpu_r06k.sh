# r06: the small-kernel pre-load fix -- the old diag library (ab/) and the new
# one through tools/small_k_check.py, then the new bitwise tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIB=pathtracker-models_amd/ptamd/ab/libptcell_olddiag.so timeout -k 10 200 python -u tools/small_k_check.py > gpurun_out/r06k_old.txt 2>&1
r=$?; echo "old:"; grep "k=" gpurun_out/r06k_old.txt; [ $r -eq 0 ] || { tail -5 gpurun_out/r06k_old.txt; exit $r; }
timeout -k 10 200 python -u tools/small_k_check.py > gpurun_out/r06k_new.txt 2>&1
r=$?; echo "new:"; grep "k=" gpurun_out/r06k_new.txt; [ $r -eq 0 ] || { tail -5 gpurun_out/r06k_new.txt; exit $r; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06k_tests.log 2>&1
r=$?; tail -4 gpurun_out/r06k_tests.log; exit $r
