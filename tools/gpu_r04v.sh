# r04: k_pw_bb2 staggered start of each CU's second workgroup (diagnostic
# ablate bits 24-27 = us of delay), interleaved in one process.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
MASKS="0,16777216,33554432,67108864,134217728" ROUNDS=3 timeout -k 10 300 python tools/ablate.py > gpurun_out/v_ablate.txt 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/v_ablate.txt | tail -9; exit $r
