# dword vs 2-B bf16 loads: determinism + kernel times (gpu_detvar.sh), then the
# -m gpu suite on the in-tree library.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "host $(hostname)"
ABL=1 REPS=${REPS:-4} bash tools/gpu_detvar.sh || exit $?
timeout -k 10 1000 python -u -m pytest ${SEL:-tests} -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -rf > gpurun_out/r03_gpu_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -12 gpurun_out/r03_gpu_tests.log
