#!/bin/bash
# Seven waves per SIMD, priced: the default build (ab_w6) against one compiled
# for seven (ab_w7: 72 VGPRs, a few spills), alternated, on the cover scene
# at grid 9 (327 bodies: its LDS image lets 7 workgroups share a CU) and
# grid 11 (C1's 484: LDS caps both at 6, so only the spills differ).
#   tools/gpu_w7.sh OUT [ROUNDS]
set -u
OUT=${1:?outdir}; R=${2:-2}; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/raytracing-clj_amd/lib
for r in $(seq 1 $R); do
  for g in 9 11; do
    for b in w6 w7; do
      RTCLJ_LIBRARY=$L/ab_$b.so timeout -k 10 120 python tools/scene_time.py --grid $g --frames 20 > $OUT/${b}_g${g}_$r.json 2> $OUT/${b}_g${g}_$r.err
      rc=$?; if [ $rc -ne 0 ]; then echo "$b grid $g rc=$rc"; tail -20 $OUT/${b}_g${g}_$r.err; exit $rc; fi
      echo "round $r $(cat $OUT/${b}_g${g}_$r.json)"
    done
  done
done
