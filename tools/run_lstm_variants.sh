# On the GPU box: ConvLSTM cfg3 bench of each exp/libptlstm_*.so variant in turn.
set -o pipefail
export TMPDIR=/tmp
cp pathtracker-models_amd/ptamd/libptlstm.so /tmp/libptlstm_base.so
for r in $(seq ${ROUNDS:-2}); do
  for v in exp/libptlstm_*.so; do
    cp "$v" pathtracker-models_amd/ptamd/libptlstm.so
    echo "== $v round $r"
    timeout -k 10 200 python tools/bench_convlstm.py --video --frames 64 --filt 7 --no-cpu-baseline --steps 5 2>/dev/null | cut -c1-200 || exit 1
  done
done
cp /tmp/libptlstm_base.so pathtracker-models_amd/ptamd/libptlstm.so
