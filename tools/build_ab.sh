#!/bin/bash
# Build cell-library A/B variants (compile-time switches) into ptamd/ab/, where
# tools/libab.py finds them beside the release library:
#   tools/build_ab.sh name1="-DFOO=1" name2="-DFOO=2 -DBAR=0" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p pathtracker-models_amd/ptamd/ab
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -fPIC -shared \
    -DPT_SRC_HASH="\"ab-$name\"" $flags -I include -o pathtracker-models_amd/ptamd/ab/libptcell_$name.so \
    pathtracker-models_amd/csrc/pt_cell.hip pathtracker-models_amd/csrc/pt_readout.hip 2>/dev/null &
done
wait
ls -la pathtracker-models_amd/ptamd/ab/
