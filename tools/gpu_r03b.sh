# Round-3 A/B on the GPU box: every exp/libptcell_*.so variant swapped in as the
# package library -> determinism_check.py (bitwise run-to-run) + ablate.py
# (per-launch kernel times, fused vs split forward); then the in-tree library is
# restored and (unless NOTESTS) the -m gpu suite runs.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cp pathtracker-models_amd/ptamd/libptcell.so /tmp/libptcell_base.so
for v in exp/libptcell_*.so; do
  cp "$v" pathtracker-models_amd/ptamd/libptcell.so
  echo "== $v"
  timeout -k 10 120 python tools/determinism_check.py > gpurun_out/det_$(basename $v .so).log 2>&1
  r=$?; grep -E "^(bf16|f32)" gpurun_out/det_$(basename $v .so).log | cut -c1-300; [ $r -eq 0 ] || { tail -5 gpurun_out/det_$(basename $v .so).log; exit $r; }
  MASKS=${MASKS:-"0:PT_CELL_FUSED=0,0:PT_CELL_FUSED=1"} ROUNDS=${ROUNDS:-2} timeout -k 10 200 python tools/ablate.py > gpurun_out/abl_$(basename $v .so).log 2>&1
  r=$?; grep -v amdgpu.ids gpurun_out/abl_$(basename $v .so).log | tail -4; [ $r -eq 0 ] || exit $r
done
cp /tmp/libptcell_base.so pathtracker-models_amd/ptamd/libptcell.so
[ -n "$NOTESTS" ] && exit 0
timeout -k 10 1000 python -u -m pytest ${SEL:-tests} -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -rf > gpurun_out/r03_gpu_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -25 gpurun_out/r03_gpu_tests.log
