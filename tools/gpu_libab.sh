# A/B of the cell-library builds in ptamd/ab/ against the release library
# (tools/libab.py, one process, interleaved): TAG names the output.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-5} timeout -k 10 400 python -u tools/libab.py > gpurun_out/${TAG:-ab}_libab.txt 2>&1
r=$?; echo LIBAB_EXIT $r; grep -v amdgpu.ids gpurun_out/${TAG:-ab}_libab.txt; exit $r
