# Run-to-run determinism (tools/det_locate.py, headline size) for the in-tree
# library and every exp/libptcell_*.so variant swapped in; restores the
# in-tree library at the end.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cp pathtracker-models_amd/ptamd/libptcell.so /tmp/libptcell_base.so
for v in /tmp/libptcell_base.so exp/libptcell_*.so; do
  cp "$v" pathtracker-models_amd/ptamd/libptcell.so
  n=$(basename $v .so)
  REPS=${REPS:-4} timeout -k 10 200 python -u tools/det_locate.py > gpurun_out/dl_$n.log 2>&1
  r=$?
  echo "== $n: $(grep -c '"frames": \[\]' gpurun_out/dl_$n.log) clean of $(grep -c saved_equal gpurun_out/dl_$n.log)"
  [ $r -eq 0 ] || { tail -5 gpurun_out/dl_$n.log; exit $r; }
  if [ -n "$ABL" ]; then
    MASKS=${MASKS:-"0:PT_CELL_FUSED=0,0:PT_CELL_FUSED=1"} ROUNDS=2 timeout -k 10 200 python tools/ablate.py > gpurun_out/abl_$n.log 2>&1
    r=$?; grep -v amdgpu.ids gpurun_out/abl_$n.log | tail -3; [ $r -eq 0 ] || exit $r
  fi
done
cp /tmp/libptcell_base.so pathtracker-models_amd/ptamd/libptcell.so
