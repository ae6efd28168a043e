# r06: the conv-loop micro-benchmark (tools/micro/conv_loop.hip) and the HW_ID
# phase trace at HEAD (tools/trace.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/conv_loop > gpurun_out/r06f_conv_loop.txt 2>&1
r=$?; echo MICRO_EXIT $r; cat gpurun_out/r06f_conv_loop.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 60 ./tools/micro/conv_loop_nowr > gpurun_out/r06f_conv_loop_nowr.txt 2>&1
r=$?; echo MICRO_NOWR_EXIT $r; cat gpurun_out/r06f_conv_loop_nowr.txt; [ $r -eq 0 ] || exit $r
TAG=r06f timeout -k 10 200 python -u tools/trace.py > gpurun_out/r06f_trace.txt 2>&1
r=$?; echo TRACE_EXIT $r; exit $r
