# r04: k_wgrad16 (16-wave weight gradients) -- A/B test against the 8-wave
# kernel, then the bench with PT_WG16=1 (default) and PT_WG16=0.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgrad16.py > gpurun_out/l_tests.log 2>&1
r=$?; tail -8 gpurun_out/l_tests.log; [ $r -eq 0 ] || exit $r
for v in 1 0 1 0; do
  PT_WG16=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/l_bench_$v.json 2> gpurun_out/l_bench_$v.err
  r=$?; echo "WG16=$v exit $r"; python3 -c "import json; d=json.load(open('gpurun_out/l_bench_$v.json')); print(d['value'], d['ms_per_step'], d['kernels_ms_per_step']['k_wgrad'])"; [ $r -eq 0 ] || { tail -5 gpurun_out/l_bench_$v.err; exit $r; }
done
