set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -x > gpurun_out/parity4.log 2>&1
echo PYTEST_EXIT $?
tail -30 gpurun_out/parity4.log
timeout -k 10 300 python tools/ablate.py > gpurun_out/ablate4.log 2>&1
echo ABL_EXIT $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench4.json 2> gpurun_out/bench4.err
echo EXIT $?
cat gpurun_out/ablate4.log; cat gpurun_out/bench4.json; tail -3 gpurun_out/bench4.err
