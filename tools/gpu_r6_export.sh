#!/bin/bash
# Round 6: path export for split launches (RTCLJ_EXPORT=1 export + sweep,
# 2 relay): the parity tests, then C1's shards with and without it
# (tools/shard_time.py, alternated configs), export limits and split rounds.
#   tools/gpu_r6_export.sh OUT [MODE]
set -u
OUT=${1:?outdir}; M=${2:-1}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_export.py tests/test_gpu_schedule.py tests/test_gpu_compact.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | head -20; exit $rc; }
timeout -k 10 600 python -u tools/shard_time.py --workload c1 --worlds 1 2 4 8 --reps 9 \
  --configs "" "RTCLJ_EXPORT=$M" "RTCLJ_EXPORT=$M,RTCLJ_EXPORT_LIM=32" "RTCLJ_EXPORT=$M,RTCLJ_EXPORT_LIM=16" "" "RTCLJ_EXPORT=$M" \
  > "$OUT/shard_c1_export.txt" 2>&1
rc=$?; echo "shard rc=$rc"; grep -E "config|N=" "$OUT/shard_c1_export.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/shard_time.py --workload c1 --worlds 8 --reps 9 \
  --configs "RTCLJ_EXPORT=$M,RTCLJ_SPLIT_ROUNDS=2" "RTCLJ_EXPORT=$M,RTCLJ_SPLIT_ROUNDS=4" "RTCLJ_EXPORT=$M,RTCLJ_SPLIT_ROUNDS=6" "" \
  > "$OUT/shard_c1_export_rounds.txt" 2>&1
rc=$?; echo "rounds rc=$rc"; grep -E "config|N=" "$OUT/shard_c1_export_rounds.txt"; exit $rc
