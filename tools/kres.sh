#!/bin/bash
# Register / spill / LDS report of the kernels in one HIP source (compile-only):
#   bash tools/kres.sh katacoffee_amd/csrc/nn.hip [extra hipcc flags]
src=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -I"$(dirname "$src")" "$@" -c "$src" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Name:/ {n=$NF; sub(/\[.*/, "", n); name=$0; sub(/.*Name: /, "", name); sub(/ \[.*/, "", name)}
       /VGPRs:/ {v=$0; sub(/.*VGPRs: /, "", v); sub(/ .*/, "", v)}
       /VGPRs Spill:/ {sp=$0; sub(/.*Spill: /, "", sp); sub(/ .*/, "", sp)}
       /LDS Size/ {l=$0; sub(/.*block\]: /, "", l); sub(/ .*/, "", l); printf "%-90.90s vgpr %4s spill %4s lds %s\n", name, v, sp, l}'
