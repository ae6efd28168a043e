# Bench A/B of cell-library builds on one box, alternating: bench.py (headline)
# with the release library and with ptamd/ab/libptcell_${B}.so in its place;
# with HB set, tools/bench_hgru.py (cfg4) the same way with libptcell_${HB}.so.
# Optional SEL: GPU tests run first (pytest -k SEL).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=pathtracker-models_amd/ptamd
if [ -n "$SEL" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -k "$SEL" -v -m gpu -p no:cacheprovider -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  r=$?; echo PYTEST_EXIT $r; tail -3 gpurun_out/${TAG}_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_tests.log | head -20; exit $r; }
fi
cp $L/libptcell.so /tmp/rel.so
for i in 1 2; do
  for v in rel ${B}; do
    if [ $v = rel ]; then cp /tmp/rel.so $L/libptcell.so; else cp $L/ab/libptcell_$v.so $L/libptcell.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_bench_${v}_$i.json 2> gpurun_out/${TAG}_bench_${v}_$i.err
    r=$?; echo "BENCH $v $i EXIT $r"; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench_${v}_$i.err; cp /tmp/rel.so $L/libptcell.so; exit $r; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'])"
  done
done
if [ -n "$HB" ]; then
  for v in rel ${HB}; do
    if [ $v = rel ]; then cp /tmp/rel.so $L/libptcell.so; else cp $L/ab/libptcell_$v.so $L/libptcell.so; fi
    timeout -k 10 300 python tools/bench_hgru.py --steps 5 --warmup 2 > gpurun_out/${TAG}_hgru_${v}.json 2> gpurun_out/${TAG}_hgru_${v}.err
    r=$?; echo "HGRU $v EXIT $r"; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_hgru_${v}.err; cp /tmp/rel.so $L/libptcell.so; exit $r; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_hgru_${v}.json')); print('hgru $v', d['value'], d['ms_per_step'], d['kernels_ms_per_step'])"
  done
fi
cp /tmp/rel.so $L/libptcell.so
