#!/bin/bash
# Code size (bytes) and register use of a specialised kernel variant compiled
# offline like hipRTC does: scripts/spec_size.sh "<defines>" [lds bvh csg quads]
# (the render kernel's hot loop must stay within the 64 KB instruction cache
# two CUs share)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
D=${TMPDIR:-/tmp}/spec_size.$$
mkdir -p $D
printf '#include "rt_render.h"\ntemplate __global__ void rt_render_kernel<%s, %s, %s, %s>(const char*, Params);\n' \
  ${2:-true} ${3:-false} ${4:-false} ${5:-false} > $D/spec.hip
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$R/include -I$R/go-raytracer_amd/csrc --cuda-device-only"
/opt/rocm/bin/hipcc $F -o $D/spec.co $D/spec.hip $1 2>/dev/null
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$D/spec.co --output=$D/spec.elf \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950
/opt/rocm/lib/llvm/bin/llvm-readelf -s $D/spec.elf | awk '$4 == "FUNC" && $8 ~ /rt_render_kernel/ {print "kernel_bytes", $3}' | head -1
/opt/rocm/bin/hipcc $F -S -o $D/spec.s $D/spec.hip $1 2>/dev/null
grep -E "^\s+\.(vgpr_count|vgpr_spill_count|sgpr_spill_count):" $D/spec.s | sort | uniq | tr -s ' ' | tr '\n' ' '; echo
rm -rf $D
