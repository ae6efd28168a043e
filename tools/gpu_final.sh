# Round measurement on the GPU box (TAG names the outputs): GPU tests, smoke,
# rocprofv3 kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes -> the PMC
# traffic summary stamped with the library's source hash, then the bench line
# LAST so that its roofline.traffic comes from that summary.  Stops at the
# first failing step; every GPU step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider -x --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -2 gpurun_out/${TAG}_tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_tests.log | head -30; exit $r; }
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1
r=$?; echo SMOKE_EXIT $r; tail -1 gpurun_out/${TAG}_smoke.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_prof.log 2>&1
r=$?; echo PROF_EXIT $r; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_prof.log; exit $r; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmca -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_pmca.log 2>&1
r=$?; echo PMCA_EXIT $r; [ $r -eq 0 ] || exit $r
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmcb -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32 > gpurun_out/${TAG}_pmcb.log 2>&1
r=$?; echo PMCB_EXIT $r; [ $r -eq 0 ] || exit $r
python tools/pmc_traffic.py gpurun_out/${TAG}_pmca gpurun_out/${TAG}_pmcb gpurun_out/${TAG}_pmc_traffic.json "B=256 T=64 bf16" > gpurun_out/${TAG}_pmc.txt 2>&1
r=$?; echo PMC_SUMMARY_EXIT $r; [ $r -eq 0 ] || exit $r
cp gpurun_out/${TAG}_pmc_traffic.json profiles/${TAG}_pmc_traffic.json   # (this box's copy of the tree) for the bench line below
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/${TAG}_bench.json; [ $r -eq 0 ] || tail -8 gpurun_out/${TAG}_bench.err
exit $r
