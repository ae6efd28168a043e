# r06: the N>1 bench step rehearsed on a one-GPU box (bench.py --rehearse:
# 2 ranks on cuda:0 over gloo, the three-part gradient exchange) and the
# 2-process GPU dist tests; every GPU step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --rehearse \
  > gpurun_out/r06r_bench2.txt 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/r06r_bench2.txt | tail -5; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r06r_dist.log 2>&1
r=$?; tail -8 gpurun_out/r06r_dist.log; exit $r
