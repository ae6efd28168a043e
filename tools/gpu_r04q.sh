# r04: k_wgrad16 LDS-DMA staging on tiled (64x64) frames: A/B test, then the
# cfg4 bench with PT_WGDMA=1 (default) and 0.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgrad16.py > gpurun_out/q_tests.log 2>&1
r=$?; tail -6 gpurun_out/q_tests.log; [ $r -eq 0 ] || exit $r
for v in 1 0; do
  PT_WGDMA=$v timeout -k 10 400 python tools/bench_hgru.py --cpu-seconds 3 > gpurun_out/q_hgru_$v.json 2> gpurun_out/q_hgru_$v.err
  r=$?; echo "WGDMA=$v exit $r"; python3 -c "import json; d=json.load(open('gpurun_out/q_hgru_$v.json')); print(d['value'], d['ms_per_step'], d['kernels_ms_per_step']['k_wgrad'])"; [ $r -eq 0 ] || { tail -5 gpurun_out/q_hgru_$v.err; exit $r; }
done
