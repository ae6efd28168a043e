# Determinism of each exp/libptcell_*.so variant (tools/determinism_check.py at
# B, T): bitwise run-to-run per parameter gradient.  The in-tree library is
# restored at the end.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cp pathtracker-models_amd/ptamd/libptcell.so /tmp/libptcell_base.so
for v in exp/libptcell_*.so; do
  n=$(basename $v .so)
  cp "$v" pathtracker-models_amd/ptamd/libptcell.so
  B=${B:-256} T=${T:-64} timeout -k 10 200 python tools/determinism_check.py > gpurun_out/vd_${n}.log 2>&1
  r=$?; echo "== $n"; grep -E "^(bf16|f32)" gpurun_out/vd_${n}.log | cut -c1-240; [ $r -eq 0 ] || { tail -3 gpurun_out/vd_${n}.log; exit $r; }
done
cp /tmp/libptcell_base.so pathtracker-models_amd/ptamd/libptcell.so
