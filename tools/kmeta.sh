#!/bin/bash
# kmeta.sh OBJ [REGEX]: register / scratch / LDS metadata of the gfx950 kernels in
# a hipcc object (the .hip_fatbin bundle), one line per kernel
set -e
t=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$1" $t/fb.bin
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$t/fb.bin \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/dev.elf
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $t/dev.elf | \
    grep -E "^\s+\.name:|\.vgpr_count|\.agpr_count|private_segment_fixed_size|vgpr_spill_count|group_segment_fixed" | \
    paste - - - - - - | sed 's/  */ /g; s/\t/ /g' | grep -E "${2:-.}" || true
rm -rf $t
