# Same-box network-only A/B of library variants (tools/build_variant.sh):
#   bash tools/ab_nn.sh PRECISION VARIANT...   (main = the in-tree library)
prec=$1; shift
for v in "$@"; do
  if [ $v = main ]; then unset KATACOFFEE_LIB; else export KATACOFFEE_LIB=tools/_build/libkatacoffee_$v.so; fi
  echo "== $v"
  timeout -k 10 120 python tools/nn_bench.py --precision $prec --n 960,1024,2048 --iters 50
done
