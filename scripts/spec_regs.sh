#!/bin/bash
# Register use of a specialised kernel variant, compiled offline like hipRTC
# does at run time: scripts/spec_regs.sh "<defines>" [lds bvh csg quads]
# e.g. C3: scripts/spec_regs.sh "-DRT_SPEC_KMASK=15 -DRT_SPEC_FEAT=0 -DRT_SPEC_NOBJ=4 -DRT_SPEC_KINDS=1,3,2,0 -DRT_SPEC_NLIGHTS=4 -DRT_SPEC_POWBITS=6"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
D=${TMPDIR:-/tmp}/spec_regs.$$
mkdir -p $D
printf '#include "rt_render.h"\ntemplate __global__ void rt_render_kernel<%s, %s, %s, %s>(const char*, Params);\n' \
  ${2:-true} ${3:-false} ${4:-false} ${5:-false} > $D/spec.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$R/include -I$R/go-raytracer_amd/csrc \
  --cuda-device-only -S -o $D/spec.s $D/spec.hip $1
grep -E "^\s+\.(vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|agpr_count):" $D/spec.s | sort | uniq
rm -rf $D
