#!/bin/bash
# Split-launch occupancy A/B: shard timings (1 and 8 ranks) of the product
# library and of a candidate build, alternated:  tools/gpu_r5q6.sh OUT lib
set -u
OUT=$1; L=$2; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python tools/shard_time.py --workload c1 --worlds 1 8 --reps 9 --inflight 2 --frames 60 > "$OUT/base_$r.log" 2>&1 || exit $?
  grep "N=" "$OUT/base_$r.log" | sed "s/^/base $r /"
  RTCLJ_LIBRARY=$PWD/$L timeout -k 10 200 python tools/shard_time.py --workload c1 --worlds 1 8 --reps 9 --inflight 2 --frames 60 > "$OUT/cand_$r.log" 2>&1 || exit $?
  grep "N=" "$OUT/cand_$r.log" | sed "s/^/cand $r /"
done
