#!/bin/bash
# A/B variant of libkatacoffee.so with extra defines, for same-box comparisons
# (KATACOFFEE_LIB=tools/_build/libkatacoffee_NAME.so python bench.py ...):
#   bash tools/build_variant.sh NAME -DSOME_SWITCH=1 ...
set -e
name=$1; shift
cd "$(dirname "$0")/../katacoffee_amd/csrc"
out=_build/var_$name
mkdir -p $out ../../tools/_build
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-result $*"
ls *.hip *.cpp | grep -v cli_selfplay | xargs -P 8 -I{} sh -c \
  'f={}; case $f in *.cpp) x="-x hip";; *) x="";; esac; /opt/rocm/bin/hipcc '"$FLAGS"' $x -c $f -o '"$out"'/${f%.*}.o'
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/libkatacoffee_$name.so $out/*.o -Wl,--no-undefined
echo built tools/_build/libkatacoffee_$name.so
