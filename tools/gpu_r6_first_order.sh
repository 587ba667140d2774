#!/bin/bash
# Round 6: a shape's first launch bottom-up (RTCLJ_FIRST_ORDER=1) against
# row-major: tools/first_frame.py (new-shape launches, alternated with the
# schedule off) under each setting, and the bench line's dispatch_order leg.
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for F in 0 1; do
    RTCLJ_FIRST_ORDER=$F timeout -k 10 300 python -u tools/first_frame.py --workload c1 --rounds 9 --json "$OUT/ff_r${r}_f$F.json" > "$OUT/ff_r${r}_f$F.txt" 2>&1 || exit $?
    echo "round $r first_order $F: $(grep 'first frame' $OUT/ff_r${r}_f$F.txt)"
  done
done
