# r04: k_wgrad16 LDS-DMA form, phase ablation (64: no MFMA body, 128: no DMAs).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
MASKS="0,64,128,192" ROUNDS=2 timeout -k 10 300 python tools/ablate.py > gpurun_out/o_ablate.txt 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/o_ablate.txt | tail -8; exit $r
