# r04: hGRU k_pw_bb2 with 2 sets (bf16): hGRU + pwb2 parity tests, then the
# cfg4 bench with PT_PWB2=1 (default) and PT_PWB2=0.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pwb2.py $(ls tests/test_gpu_*hgru*.py) > gpurun_out/k_tests.log 2>&1
r=$?; tail -3 gpurun_out/k_tests.log; [ $r -eq 0 ] || exit $r
for v in 1 0; do
  PT_PWB2=$v timeout -k 10 400 python tools/bench_hgru.py --cpu-seconds 3 > gpurun_out/k_hgru_$v.json 2> gpurun_out/k_hgru_$v.err
  r=$?; echo "PWB2=$v exit $r"; cut -c1-400 gpurun_out/k_hgru_$v.json; [ $r -eq 0 ] || { tail -5 gpurun_out/k_hgru_$v.err; exit $r; }
done
