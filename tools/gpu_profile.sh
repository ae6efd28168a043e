# Round profile: full bench line (with CPU baseline), rocprofv3 kernel trace + stats,
# FETCH_SIZE / WRITE_SIZE passes -> per-kernel HBM traffic.  TAG names the outputs.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
python __graft_entry__.py build > gpurun_out/${TAG}_build.log 2>&1 || { echo BUILD_FAIL; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/${TAG}_bench.json; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $r; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
r=$?; echo PROF_EXIT $r; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_prof.log; exit $r; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmca -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_pmca.log 2>&1
r=$?; echo PMCA_EXIT $r; [ $r -eq 0 ] || exit $r
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmcb -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_pmcb.log 2>&1
r=$?; echo PMCB_EXIT $r; [ $r -eq 0 ] || exit $r
python tools/pmc_traffic.py gpurun_out/${TAG}_pmca gpurun_out/${TAG}_pmcb gpurun_out/${TAG}_pmc_traffic.json "B=256 T=64 bf16"
