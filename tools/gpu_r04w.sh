# r04: k_wgrad16 smallest-shape tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgrad16.py > gpurun_out/w_tests.log 2>&1
r=$?; tail -12 gpurun_out/w_tests.log; exit $r
