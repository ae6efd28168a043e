#!/bin/bash
# Per-kernel VGPR/AGPR/spill/occupancy of the gfx950 build (compile-time only).
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -fPIC -c -I/root/repo/include \
  /root/repo/pathtracker-models_amd/csrc/pt_cell.hip -o /tmp/ptc_res.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: //p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name/{if(n)print line; n=$3; line=n; next} /VGPRs:|AGPRs:|VGPRs Spill|Occupancy|LDS Size/{line=line" | "$0} END{print line}' |
  c++filt | sed 's/ptc:://; s/CellArgs<[^>]*>//; s/ConvArgs<[^>]*>//'
