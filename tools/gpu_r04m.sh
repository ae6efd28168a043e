# r04: k_wgrad phase ablation (64: no MFMA body, 128: no band loads), the
# 16-wave and the 8-wave form, interleaved in one process.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
MASKS="0,64,128,192,0:PT_WG16=0,64:PT_WG16=0,128:PT_WG16=0" ROUNDS=2 timeout -k 10 300 python tools/ablate.py > gpurun_out/m_ablate.txt 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/m_ablate.txt | tail -30; exit $r
