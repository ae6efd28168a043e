set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -x > gpurun_out/parity5.log 2>&1
echo PYTEST_EXIT $?
tail -5 gpurun_out/parity5.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err
echo BENCH_EXIT $?
cat gpurun_out/bench5.json
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
echo LIST_EXIT $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc5a -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc5a.log 2>&1
echo PMC_A $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc5b -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc5b.log 2>&1
echo PMC_B $?
