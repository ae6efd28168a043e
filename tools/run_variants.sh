# On the GPU box: per-launch kernel times of each exp/libptcell_*.so variant,
# run in turn ROUNDS times (tools/ablate.py; each variant swapped in as the
# package's library), stopping at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cp pathtracker-models_amd/ptamd/libptcell.so /tmp/libptcell_base.so; cp pathtracker-models_amd/ptamd/libptcell_diag.so /tmp/libptcell_diagbase.so
for r in $(seq ${ROUNDS:-2}); do
  for v in exp/libptcell_*.so; do
    cp "$v" pathtracker-models_amd/ptamd/libptcell.so; cp "$v" pathtracker-models_amd/ptamd/libptcell_diag.so
    echo "== $v round $r"
    MASKS=0 ROUNDS=2 timeout -k 10 200 python tools/ablate.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
  done
done
cp /tmp/libptcell_base.so pathtracker-models_amd/ptamd/libptcell.so; cp /tmp/libptcell_diagbase.so pathtracker-models_amd/ptamd/libptcell_diag.so
