# end-to-end harness throughput on synthetic GZIP TFRecord shards (reader + H2D + step)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_harness.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/p_h.log 2>&1
r=$?; tail -2 gpurun_out/p_h.log; [ $r -eq 0 ] || exit $r
PT_CELL_DTYPE=${PT_CELL_DTYPE:-bf16} timeout -k 10 500 python -u pathtracker-models_amd/mainclean.py --model InT --name pipe --dist 14 --speed 1 --length 64 -b 256 --epochs 1 --print-freq 1 --data-root /tmp/pt_shards --synthetic 12288 --results-root /tmp/pt_res --max-iters 40 > gpurun_out/pipeline.log 2>&1
r=$?; echo PIPE_EXIT $r; grep -E "^Epoch" gpurun_out/pipeline.log | tail -3 | cut -c1-150; exit $r
