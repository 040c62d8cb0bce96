#!/bin/bash
# Per-kernel register / spill / occupancy summary of one HIP source (gfx950), e.g.
#   scripts/regs.sh poi_recommendation_models_amd/csrc/nais_train.hip [extra hipcc flags]
src=$(readlink -f "$1"); shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize \
  -I /root/repo/include -c "$src" -o /tmp/regs_probe.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  grep -E "Name:|VGPRs:|AGPRs:|Spill:|Occupancy" | sed -E 's/.*remark: *//; s/ \[-Rpass.*//' |
  awk '/Function Name:/{if(l)print l; l=$3; next}{sub(/^ +/,""); l=l" | "$0}END{print l}' | c++filt
