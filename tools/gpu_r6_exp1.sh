#!/bin/bash
# Round 6 experiments: variant 28's split rounds and frames in flight on C1's
# shards (tools/shard_time.py), and the first frame (tools/first_frame.py).
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/shard_time.py --workload c1 --worlds 1 4 8 --reps 9 \
  --configs "RTCLJ_TH4=0" "" "RTCLJ_TH4_SPLIT_ROUNDS=2" "RTCLJ_TH4_SPLIT_ROUNDS=3" "RTCLJ_TH4=0" > "$OUT/shard_c1_th4.txt" 2>&1
rc=$?; echo "shard rc=$rc"; grep -E "config|N=" "$OUT/shard_c1_th4.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/shard_time.py --workload c1 --worlds 1 8 --reps 5 --inflight 2 --frames 40 \
  --configs "RTCLJ_TH4=0" "" > "$OUT/shard_c1_th4_inflight.txt" 2>&1
rc=$?; echo "inflight rc=$rc"; grep -E "config|N=" "$OUT/shard_c1_th4_inflight.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/first_frame.py --workload c1 --rounds 9 --cold --json "$OUT/first_frame.json" > "$OUT/first_frame.txt" 2>&1
rc=$?; echo "first rc=$rc"; cat "$OUT/first_frame.txt" | grep -v amdgpu.ids; exit $rc
