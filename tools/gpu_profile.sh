# Round profile: full bench line (with CPU baseline), rocprofv3 kernel trace + stats,
# FETCH_SIZE / WRITE_SIZE passes -> per-kernel HBM traffic.  TAG names the outputs.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
# libraries are prebuilt in-tree (python __graft_entry__.py build on the CPU side)
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
r=$?; echo BENCH_EXIT $r; cat gpurun_out/${TAG}_bench.json; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $r; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
r=$?; echo PROF_EXIT $r; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_prof.log; exit $r; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmca -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_pmca.log 2>&1
r=$?; echo PMCA_EXIT $r; [ $r -eq 0 ] || exit $r
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmcb -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_pmcb.log 2>&1
r=$?; echo PMCB_EXIT $r; [ $r -eq 0 ] || exit $r
python tools/pmc_traffic.py gpurun_out/${TAG}_pmca gpurun_out/${TAG}_pmcb gpurun_out/${TAG}_pmc_traffic.json "B=256 T=64 bf16"
# end-to-end harness throughput on synthetic GZIP TFRecord shards (reader + H2D + step)
timeout -k 10 400 python -u pathtracker-models_amd/mainclean.py --model InT --name pipe --dist 14 --speed 1 --length 64 -b 256 --epochs 1 --print-freq 1 --data-root /tmp/pt_shards --synthetic 4096 --results-root /tmp/pt_res --max-iters 14 > gpurun_out/${TAG}_pipeline.log 2>&1
r=$?; echo PIPE_EXIT $r; grep -E "^Epoch" gpurun_out/${TAG}_pipeline.log | tail -4 | cut -c1-160
