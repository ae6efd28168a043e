# determinism at the headline size, in-tree library; then the same with the
# split forward; stops at the first failure
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B=256 T=64 timeout -k 10 300 python tools/determinism_check.py > gpurun_out/det_b256.log 2>&1
r=$?; cut -c1-600 gpurun_out/det_b256.log | grep -v amdgpu; [ $r -eq 0 ] || exit $r
PT_CELL_FUSED=0 B=256 T=64 timeout -k 10 300 python tools/determinism_check.py > gpurun_out/det_b256_split.log 2>&1
r=$?; cut -c1-600 gpurun_out/det_b256_split.log | grep -v amdgpu; [ $r -eq 0 ] || exit $r
MASKS="0:PT_CELL_FUSED=0,0:PT_CELL_FUSED=1" ROUNDS=2 timeout -k 10 200 python tools/ablate.py > gpurun_out/abl_fused.log 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/abl_fused.log | tail -4
