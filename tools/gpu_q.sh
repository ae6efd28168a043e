set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -q -m gpu -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/q_parity.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -3 gpurun_out/q_parity.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/q_parity.log | head -20; exit $r; }
MASKS=${MASKS:-0,4} ROUNDS=3 timeout -k 10 300 python tools/ablate.py > gpurun_out/q_ablate.log 2>&1
r=$?; echo ABL_EXIT $r; cat gpurun_out/q_ablate.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err
r=$?; echo BENCH_EXIT $r; python -c "import json;d=json.load(open('gpurun_out/q_bench.json'));print(d['value'],d['ms_per_step'],d['kernels_ms_per_step'])"; [ $r -eq 0 ] || tail -5 gpurun_out/q_bench.err
