set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
echo EXIT $?
cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
