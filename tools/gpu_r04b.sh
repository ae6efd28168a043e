# r04: locate the -ffp-contract=on bf16 divergence (the contract diagnostic
# build, backward stopped after 5 launches, per-element records of the
# differing k_pw_ba outputs).  Every GPU step under its own limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=pathtracker-models_amd/ptamd
cp $L/libptcell_diag.so /tmp/diag.so
cp exp/libptcell_contractdiag.so $L/libptcell_diag.so
PT_CELL_DEBUG_STOP=5 EXPLAIN_T=62 B=256 T=64 REPS=6 timeout -k 10 300 python -u tools/det_locate.py > gpurun_out/b_detloc5.log 2>&1
r=$?; echo DETLOC_EXIT $r; cut -c1-300 gpurun_out/b_detloc5.log | grep -v amdgpu.ids
cp /tmp/diag.so $L/libptcell_diag.so
exit $r
