#!/bin/bash
# Build experimental libptcell variants (compile-time switches) into exp/:
#   tools/build_variants.sh name1="-DFOO=1" name2="-DFOO=2" ...
# tools/run_variants.sh times each on the GPU box (tools/ablate.py).
set -e
cd "$(dirname "$0")/.."
mkdir -p exp
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -fPIC -shared -DPT_SRC_HASH="\"exp-$name\"" $flags \
    -I include -o exp/libptcell_$name.so pathtracker-models_amd/csrc/pt_cell.hip pathtracker-models_amd/csrc/pt_readout.hip 2>/dev/null &
done
wait
ls -la exp/
