#!/bin/bash
# Register / spill counts of the megakernel instances in a trace.hip object (code-object notes).
# Usage: tools/kstats.sh [trace.hip.o] (default: the in-tree build)
obj=${1:-shirley-raytracing-rs_amd/build/rt/trace.hip.o}
tmp=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fb.bin "$obj" &&
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$tmp/fb.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$tmp/k.co &&
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $tmp/k.co | awk '
  /\.name:/ {name=$2}
  /\.sgpr_spill_count:/ {ss=$2} /\.vgpr_spill_count:/ {vs=$2} /\.vgpr_count:/ {vc=$2} /\.sgpr_count:/ {sc=$2}
  /\.private_segment_fixed_size:/ {ps=$2}
  /\.wavefront_size:/ { if (name ~ /trace_kernel/) printf "%-60s vgpr %s (spill %s) sgpr %s (spill %s) scratch %s\n", name, vc, vs, sc, ss, ps }'
rm -rf $tmp
