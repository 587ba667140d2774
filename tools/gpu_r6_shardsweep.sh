#!/bin/bash
# Round 6: C1's per-rank shard times under launch knobs (tools/shard_time.py
# --configs), the default first and last.   tools/gpu_r6_shardsweep.sh OUT
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -u tools/shard_time.py --workload c1 --worlds 1 2 4 8 --reps 7 \
  --configs "" "RTCLJ_SHARE_RECORDED=1" "RTCLJ_SHARE_RECORDED=1,RTCLJ_SPLIT=1" "RTCLJ_SPLIT_ROUNDS=2" \
            "RTCLJ_SPLIT_ROUNDS=4" "RTCLJ_THIEVES=8,RTCLJ_SHARE_RECORDED=1" "" > "$OUT/sweep.txt" 2>&1
rc=$?; grep -E "config|N=" "$OUT/sweep.txt"; exit $rc
