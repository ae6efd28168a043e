# r04 first GPU call: GPU tests on the release build, the bf16 attribution
# (diagnostic build), the -ffp-contract=on determinism evidence, a short bench.
# Stops at the first GPU fault / timeout; every GPU step under its own limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=pathtracker-models_amd/ptamd
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider -x --timeout 150 --timeout-method thread > gpurun_out/a_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/a_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/a_tests.log | head -30; exit $r; }
DIAG_PARAMS=trained timeout -k 10 300 python -u tools/bf16_attrib.py > gpurun_out/a_attrib.log 2>&1
r=$?; echo ATTRIB_EXIT $r; cut -c1-400 gpurun_out/a_attrib.log | grep -v amdgpu.ids; [ $r -eq 0 ] || exit $r
cp $L/libptcell.so /tmp/rel.so; cp $L/libptcell_diag.so /tmp/diag.so
cp exp/libptcell_contract.so $L/libptcell.so
B=256 T=64 timeout -k 10 300 python -u tools/determinism_check.py > gpurun_out/a_det_contract.log 2>&1
r=$?; echo DET_CONTRACT_EXIT $r; cut -c1-300 gpurun_out/a_det_contract.log | grep -v amdgpu.ids; [ $r -eq 0 ] || exit $r
cp /tmp/rel.so $L/libptcell.so
cp exp/libptcell_contractdiag.so $L/libptcell_diag.so
B=256 T=64 REPS=4 timeout -k 10 300 python -u tools/det_locate.py > gpurun_out/a_detloc_all.log 2>&1
r=$?; echo DETLOC_EXIT $r; cut -c1-600 gpurun_out/a_detloc_all.log | grep -v amdgpu.ids; [ $r -eq 0 ] || exit $r
cp /tmp/diag.so $L/libptcell_diag.so
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/a_bench.json 2> gpurun_out/a_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/a_bench.json; [ $r -eq 0 ] || tail -8 gpurun_out/a_bench.err
exit $r
