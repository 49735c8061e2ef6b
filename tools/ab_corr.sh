# corrected network vs the oracle's fp32 / fp16 / corrected emulations for library variants
for v in "$@"; do
  if [ $v = main ]; then unset KATACOFFEE_LIB; else export KATACOFFEE_LIB=tools/_build/libkatacoffee_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python tools/corr_debug.py 2>&1 | grep -v amdgpu.ids
done
