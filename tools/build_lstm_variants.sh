#!/bin/bash
# Build experimental libptlstm variants (compile-time switches) into exp/:
#   tools/build_lstm_variants.sh name1="-DFOO=1" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p exp
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -fPIC -shared -DPT_SRC_HASH="\"exp-$name\"" $flags \
    -I include -o exp/libptlstm_$name.so pathtracker-models_amd/csrc/pt_lstm.hip 2>/dev/null &
done
wait
ls -la exp/
