#!/bin/bash
# Round 6: C1's shards at max depth 50 / 12 / 6 / 3 (tools/shard_time.py
# --depth; not bench lines): one frame against two frames in flight, with and
# without path export.  If the single-frame tail is the latency of a launch's
# longest paths, it shrinks with the depth cap.   tools/gpu_r6_depth_tail.sh OUT
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
for D in 50 12 6 3; do
  timeout -k 10 300 python -u tools/shard_time.py --workload c1 --worlds 1 8 --reps 9 --inflight 2 --frames 40 --depth $D \
    --configs "" "RTCLJ_EXPORT=1" > "$OUT/depth$D.txt" 2>&1
  rc=$?; echo "depth $D rc=$rc"; grep -E "config|N=" "$OUT/depth$D.txt"; [ $rc -ne 0 ] && exit $rc
done
exit 0
