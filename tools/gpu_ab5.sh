#!/bin/bash
# Round-5 A/B pass: smoke (bit-exact vs the mirror) per candidate library,
# then alternated bench runs.  tools/gpu_ab5.sh OUT ROUNDS lib1 lib2 ...
set -u
OUT=$1; ROUNDS=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in "$@"; do
  RTCLJ_LIBRARY=$PWD/$L timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$(basename $L).log" 2>&1
  rc=$?; echo "smoke $L rc=$rc"; tail -2 "$OUT/smoke_$(basename $L).log"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 900 python tools/ab_libs.py --libs "$@" --rounds "$ROUNDS" --steps 20 --out "$OUT/ab.jsonl" > "$OUT/ab.log" 2>&1
rc=$?; tail -8 "$OUT/ab.log"; exit $rc
