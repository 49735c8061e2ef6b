# Same-box network-only A/B of library variants on the layered nets (C3 / C4 / C5 batch
# sizes), alternating variants twice: bash tools/ab_layered.sh PRECISION VARIANT...
prec=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = main ]; then unset KATACOFFEE_LIB; else export KATACOFFEE_LIB=tools/_build/libkatacoffee_$v.so; fi
    echo "== $v (pass $rep)"
    timeout -k 10 120 python tools/nn_bench.py --arch b10c128 --board 5 --precision $prec --n 4450 --iters 20 || exit 1
    timeout -k 10 120 python tools/nn_bench.py --arch b10c128 --board 7 --precision $prec --n 4096 --iters 10 || exit 1
    timeout -k 10 120 python tools/nn_bench.py --arch b18c384nbt --board 9 --precision $prec --n 3600 --iters 4 || exit 1
  done
done
