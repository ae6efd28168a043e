# r04: k_wgrad16 with LDS-DMA band staging: A/B test, then interleaved timing
# (DMA 16-wave / register 16-wave / 8-wave) and phase ablation of the DMA form.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgrad16.py > gpurun_out/n_tests.log 2>&1
r=$?; tail -8 gpurun_out/n_tests.log; [ $r -eq 0 ] || exit $r
MASKS="0,0:PT_WGDMA=0,0:PT_WG16=0,64,128" ROUNDS=2 timeout -k 10 300 python tools/ablate.py > gpurun_out/n_ablate.txt 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/n_ablate.txt | tail -12; exit $r
