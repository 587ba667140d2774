#!/bin/bash
# Round 5, first GPU pass: VALU instruction costs, the counter list, and the
# default bench line at HEAD on this box (baseline for the round's A/Bs).
set -u
OUT=gpurun_out/r05a
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 tools/bin/valu_cost > "$OUT/valu_cost.txt" 2>&1; rc=$?; echo "valu_cost rc=$rc"; [ $rc -ne 0 ] && exit $rc
REPO=$PWD; cd /tmp && cd "$REPO"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "list rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
echo done
