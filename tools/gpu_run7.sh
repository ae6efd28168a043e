set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -x > gpurun_out/parity7.log 2>&1
echo PYTEST_EXIT $?
tail -15 gpurun_out/parity7.log
MASKS=0,1,4,32 timeout -k 10 300 python tools/ablate.py > gpurun_out/ablate7.log 2>&1
echo ABL_EXIT $?
cat gpurun_out/ablate7.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench7.json 2> gpurun_out/bench7.err
echo BENCH_EXIT $?
cat gpurun_out/bench7.json
