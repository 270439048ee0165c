#!/bin/bash
# Per-kernel VGPR / spill / occupancy table of one HIP source (compile-only).
# usage: tools/kres.sh <file.hip> [extra hipcc flags]
f=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fgpu-flush-denormals-to-zero \
  -fdenormal-fp-math=preserve-sign -fno-slp-vectorize -Rpass-analysis=kernel-resource-usage -c "$f" -o /tmp/kres.o "$@" 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' |
  awk '/Function Name/{if(n)print line; line=$3; n=1; next} /VGPRs:|AGPRs:|Spill|Occupancy|ScratchSize/{gsub(/ +/," "); line=line" | "$0} END{print line}'
