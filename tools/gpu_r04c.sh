# r04: f32 I (headline + golden parity tests), then determinism of each
# exp/ variant (contract / contractpad / base / pad) and their kernel times.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider -x --timeout 150 --timeout-method thread > gpurun_out/c_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/c_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/c_tests.log | head -30; }
cp gpurun_out/parity_records.json gpurun_out/c_parity_records.json 2>/dev/null
bash tools/gpu_vardet.sh; r2=$?; echo VARDET_EXIT $r2; [ $r2 -eq 0 ] || exit $r2
ROUNDS=1 bash tools/run_variants.sh; r3=$?; echo VARIANTS_EXIT $r3
exit $r3
