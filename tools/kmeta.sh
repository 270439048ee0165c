# Resource usage (VGPRs, spills, LDS) of the gfx950 kernels in a hipcc object
# or device-only bundle. usage: bash tools/kmeta.sh file.o [name-substring]
set -e
f=$1; pat=${2:-.}
t=$(mktemp -d)
if /opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$t/fb $f 2>/dev/null; then b=$t/fb; else b=$f; fi
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$b --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $t/co | grep -E "^ +\.name:|\.vgpr_count|\.sgpr_count|vgpr_spill_count|group_segment_fixed_size" | paste - - - - - | sed 's/  */ /g' | grep -E "$pat" || true
rm -rf $t
