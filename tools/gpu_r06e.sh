# r06: A/B of the ptamd/ab/ builds (tools/libab.py) and the cfg4 bench
# (tools/bench_hgru.py) at the current defaults.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -k accuracy -q -m gpu -p no:cacheprovider -x --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/${TAG}_tests.log; [ $r -eq 0 ] || exit $r
ROUNDS=${ROUNDS:-5} timeout -k 10 400 python -u tools/libab.py > gpurun_out/${TAG}_libab.txt 2>&1
r=$?; echo LIBAB_EXIT $r; grep -v amdgpu.ids gpurun_out/${TAG}_libab.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u tools/bench_hgru.py --steps 5 --warmup 2 > gpurun_out/${TAG}_hgru64_bench.json 2> gpurun_out/${TAG}_hgru64_bench.err
r=$?; echo HGRU_EXIT $r; cat gpurun_out/${TAG}_hgru64_bench.json; [ $r -eq 0 ] || tail -5 gpurun_out/${TAG}_hgru64_bench.err
exit $r
