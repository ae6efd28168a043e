set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/parity2.log 2>&1
echo PYTEST_EXIT $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 10 > gpurun_out/bench2.json 2> gpurun_out/bench2.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof2.log 2>&1
echo EXIT $?
tail -3 gpurun_out/parity2.log; cat gpurun_out/bench2.json; tail -3 gpurun_out/bench2.err
