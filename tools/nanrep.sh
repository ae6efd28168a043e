# repeat the headline bench N times in fresh processes and report the final loss of each
set -o pipefail
mkdir -p gpurun_out
for i in $(seq 1 ${N:-6}); do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('run', d['value'], d['loss'], d['kernels_ms_per_step']['k_wgrad'])" || exit 1
done
