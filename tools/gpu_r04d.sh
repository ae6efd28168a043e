# r04: all GPU tests on the release build (f32 I, -fno-slp-vectorize), the
# determinism check at B=256 T=64, then kernel times of exp/ base (SLP on) vs
# noslp.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider -x --timeout 150 --timeout-method thread > gpurun_out/d_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/d_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/d_tests.log | head -30; exit $r; }
cp gpurun_out/parity_records.json gpurun_out/d_parity_records.json
B=256 T=64 timeout -k 10 300 python -u tools/determinism_check.py > gpurun_out/d_det.log 2>&1
r=$?; echo DET_EXIT $r; grep -E "^(bf16|f32)" gpurun_out/d_det.log | cut -c1-300; [ $r -eq 0 ] || exit $r
ROUNDS=2 bash tools/run_variants.sh; r3=$?; echo VARIANTS_EXIT $r3
exit $r3
