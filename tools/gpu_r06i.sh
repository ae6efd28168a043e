# r06: the fused backward A (k_conv_pw_ba) bitwise test, then the A/B of ptamd/ab/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -k "backward_a" -v -m gpu -p no:cacheprovider -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -3 gpurun_out/${TAG}_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_tests.log | head -20; exit $r; }
ROUNDS=${ROUNDS:-5} timeout -k 10 400 python -u tools/libab.py > gpurun_out/${TAG}_libab.txt 2>&1
r=$?; echo LIBAB_EXIT $r; grep -v amdgpu.ids gpurun_out/${TAG}_libab.txt; exit $r
