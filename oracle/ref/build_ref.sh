#!/bin/bash
# Builds oracle/_ref/refgen: the reference's cpp/core + cpp/game compiled from
# /root/reference as ONE translation unit together with our driver refgen.cpp.
# Nothing from the reference is copied into the repo; the sources are streamed
# through line-addressed sed fixes for the compile blockers listed in SURVEY §8(c):
#   board.cpp:220       `Loc tempSpot = loc;` redeclaration -> `tempSpot = loc.spot;`  (P3)
#   board.cpp:658       `bool suc` redeclaration            -> `suc`                   (P4)
#   boardhistory.cpp:181-183 first duplicate checkGameEnd definition deleted          (P5)
#   board.h:178 extra `Board::` qualification               -> accepted by -fpermissive (P2)
#   global.h:343-346 non-inline header globals              -> single TU (no ODR clash) (P6)
# Output: oracle/_ref/refgen (gitignored, travels to the GPU box but is only
# needed here to (re)generate tests/golden fixtures).
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
R=${KATACOFFEE_REFERENCE:-/root/reference/cpp}
OUT="$HERE/../_ref"
if [ ! -d "$R" ]; then echo "reference not present at $R; skipping"; exit 0; fi
mkdir -p "$OUT"
emit() { echo; echo "#line 1 \"$R/$1\""; if [ -n "${2:-}" ]; then sed "$2" "$R/$1"; else cat "$R/$1"; fi; }
{
  for f in core/global.cpp core/hash.cpp core/rand.cpp core/sha2.cpp core/md5.cpp core/bsearch.cpp \
           core/timer.cpp core/test.cpp core/fancymath.cpp game/graphhash.cpp; do emit $f; done
  emit game/board.cpp '220s/Loc tempSpot = loc;/tempSpot = loc.spot;/;658s/bool suc/suc/'
  emit game/boardhistory.cpp '181,183d'
  echo; echo "#line 1 \"$HERE/refgen.cpp\""; cat "$HERE/refgen.cpp"
} | g++ -std=c++17 -O2 -fpermissive -w -include "$HERE/prelude.h" -I"$R/core" -I"$R/game" -I"$R" \
      -x c++ - -o "$OUT/refgen"
echo "built $OUT/refgen"
