#!/bin/bash
# Registers, spills and scratch of every kernel in a built object (default: the
# lane kernels): bash tools/kernel_regs.sh [OBJ]
B=/opt/rocm/lib/llvm/bin
OBJ=$(readlink -f "${1:-$(dirname "$0")/../gatk-haplotypecaller-cpp17_amd/build/lane_kernel.o}")
$B/llvm-objdump --offloading "$OBJ" > /dev/null   # extracts next to the object
CO=$OBJ.0.hipv4-amdgcn-amd-amdhsa--gfx950
$B/llvm-readelf --notes "$CO" | grep -E "^ +\.name:|\.private_segment_fixed_size|\.sgpr_spill|\.vgpr_count|\.vgpr_spill" | paste - - - - - | sed 's/  */ /g'
rm -f "$CO" "$OBJ".0.host-*
