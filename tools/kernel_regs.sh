# VGPR / SGPR / LDS / scratch of the built kernels (development): kernel_regs.sh [pattern]
L=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$L/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin ${LIB:-mpi-test_amd/lib/libgsort.so}
$L/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --output=$T/g.co --targets=hipv4-amdgcn-amd-amdhsa--gfx950
$L/llvm-readelf --notes $T/g.co | grep -E "\.name:|\.private_segment_fixed_size:|\.sgpr_count:|\.vgpr_count:" | paste - - - - | sed 's/  */ /g' | grep -E "${1:-.}"
rm -rf $T
