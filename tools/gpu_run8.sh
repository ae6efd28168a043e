set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -x > gpurun_out/parity8.log 2>&1
echo PYTEST_EXIT $?
tail -3 gpurun_out/parity8.log
MASKS=0,64,128,192 timeout -k 10 300 python tools/ablate.py > gpurun_out/ablate8.log 2>&1
echo ABL_EXIT $?
cat gpurun_out/ablate8.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench8.json 2> gpurun_out/bench8.err
echo BENCH_EXIT $?
cat gpurun_out/bench8.json
