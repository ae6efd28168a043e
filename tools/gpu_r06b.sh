# r06 issue-priority A/B (PT_PRIO builds in ptamd/ab/, tools/libab.py) and the
# phase trace of the PT_PRIO=7 diagnostic build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-5} timeout -k 10 400 python -u tools/libab.py > gpurun_out/r06b_libab.txt 2>&1
r=$?; echo LIBAB_EXIT $r; grep -v amdgpu.ids gpurun_out/r06b_libab.txt; [ $r -eq 0 ] || exit $r
TAG=r06b_p7 TRACE_LIB=pathtracker-models_amd/ptamd/abdiag/libptcell_diag_p7.so timeout -k 10 200 python -u tools/trace.py > gpurun_out/r06b_trace_p7.txt 2>&1
r=$?; echo TRACE_EXIT $r; [ $r -eq 0 ] || { tail -20 gpurun_out/r06b_trace_p7.txt; exit $r; }
