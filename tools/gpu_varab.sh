# Variant A/B on the GPU box: each exp/libptcell_*.so in turn as the package
# library -> tools/ablate.py over MASKS (and, with VTESTS set, those GPU tests
# first); the in-tree library is restored at the end.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cp pathtracker-models_amd/ptamd/libptcell.so /tmp/libptcell_base.so
for v in exp/libptcell_*.so; do
  n=$(basename $v .so)
  cp "$v" pathtracker-models_amd/ptamd/libptcell.so
  echo "== $n"
  if [ -n "$VTESTS" ]; then
    timeout -k 10 300 python -u -m pytest $VTESTS -q -m gpu -p no:cacheprovider -x --timeout 150 \
      --timeout-method thread > gpurun_out/va_${n}_tests.log 2>&1
    r=$?; tail -1 gpurun_out/va_${n}_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/va_${n}_tests.log | head; exit $r; }
  fi
  MASKS=${MASKS:-0} ROUNDS=${ROUNDS:-3} timeout -k 10 200 python tools/ablate.py > gpurun_out/va_${n}.log 2>&1
  r=$?; grep -v amdgpu.ids gpurun_out/va_${n}.log | tail -n +2; [ $r -eq 0 ] || exit $r
done
cp /tmp/libptcell_base.so pathtracker-models_amd/ptamd/libptcell.so
