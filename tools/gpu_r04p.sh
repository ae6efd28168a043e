# r04: lane-linear wgrad slab stores: wgrad16 A/B + golden parity tests, then
# interleaved timing (DMA 16-wave / register 16-wave / 8-wave / skeleton).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad16.py tests/test_gpu_parity.py > gpurun_out/p_tests.log 2>&1
r=$?; tail -4 gpurun_out/p_tests.log; [ $r -eq 0 ] || exit $r
MASKS="0,0:PT_WGDMA=0,0:PT_WG16=0,192" ROUNDS=2 timeout -k 10 300 python tools/ablate.py > gpurun_out/p_ablate.txt 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/p_ablate.txt | tail -8; exit $r
