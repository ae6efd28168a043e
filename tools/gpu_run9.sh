set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/parity9.log 2>&1
r=$?; echo PYTEST_EXIT $r; [ $r -eq 0 ] || exit $r; tail -3 gpurun_out/parity9.log
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke9.log 2>&1
r=$?; echo SMOKE_EXIT $r; [ $r -eq 0 ] || exit $r; tail -2 gpurun_out/smoke9.log
timeout -k 10 300 python bench.py > gpurun_out/bench9.json 2> gpurun_out/bench9.err
r=$?; echo BENCH_EXIT $r; [ $r -eq 0 ] || exit $r; cat gpurun_out/bench9.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof9 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof9.log 2>&1
r=$?; echo PROF_EXIT $r; [ $r -eq 0 ] || exit $r; cat gpurun_out/prof9.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc9a -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc9a.log 2>&1
r=$?; echo PMCA_EXIT $r; [ $r -eq 0 ] || exit $r
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc9b -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc9b.log 2>&1
echo PMCB_EXIT $?
python tools/pmc_traffic.py gpurun_out/pmc9a gpurun_out/pmc9b gpurun_out/pmc9_traffic.json "B=256 T=64 bf16"
