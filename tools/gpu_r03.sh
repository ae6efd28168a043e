# Round-3 GPU check: the full -m gpu suite, optional probes, a short bench.
# Usage (GPU box): bash tools/gpu_r03.sh [tests-selector] ; every step has its own
# time limit and the script stops at the first failed step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -rf > gpurun_out/r03_gpu_tests.log 2>&1
r=$?; echo PYTEST_EXIT $r; tail -15 gpurun_out/r03_gpu_tests.log
[ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
if [ -n "$PROBE" ]; then
  timeout -k 10 300 python -u tools/probe_headline.py $PROBE > gpurun_out/r03_probe.log 2>&1
  r=$?; echo PROBE_EXIT $r; tail -4 gpurun_out/r03_probe.log; [ $r -eq 0 ] || exit $r
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32 \
    > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
  r=$?; echo BENCH_EXIT $r; cat gpurun_out/r03_bench.json; [ $r -eq 0 ] || tail -5 gpurun_out/r03_bench.err
fi
