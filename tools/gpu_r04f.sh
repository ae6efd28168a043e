# r04: k_pw_bb2 phase traces and ablations (diagnostic build).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PT_PWB2=1 timeout -k 10 200 python -u tools/trace.py > gpurun_out/f_trace_pwb2.log 2>&1
r=$?; echo TRACE_EXIT $r; grep -v amdgpu.ids gpurun_out/f_trace_pwb2.log | head -30; [ $r -eq 0 ] || exit $r
MASKS="0:PT_PWB2=1,16:PT_PWB2=1,8:PT_PWB2=1,32:PT_PWB2=1,56:PT_PWB2=1,512:PT_PWB2=1" ROUNDS=2 timeout -k 10 300 python -u tools/ablate.py > gpurun_out/f_ablate.log 2>&1
r=$?; echo ABLATE_EXIT $r; grep -v amdgpu.ids gpurun_out/f_ablate.log | tail -9
exit $r
