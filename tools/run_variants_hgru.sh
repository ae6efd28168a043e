# On the GPU box: hGRU cfg4 kernel times (tools/bench_hgru.py) of each
# exp/libptcell_*.so variant in turn, ROUNDS times.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cp pathtracker-models_amd/ptamd/libptcell.so /tmp/libptcell_base.so
for r in $(seq ${ROUNDS:-2}); do
  for v in exp/libptcell_*.so; do
    cp "$v" pathtracker-models_amd/ptamd/libptcell.so
    echo "== $v round $r"
    timeout -k 10 200 python tools/bench_hgru.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: round(v, 2) for k, v in d['kernels_ms_per_step'].items()})" || exit 1
  done
done
cp /tmp/libptcell_base.so pathtracker-models_amd/ptamd/libptcell.so
