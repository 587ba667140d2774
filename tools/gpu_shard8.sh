#!/bin/bash
# C1's 8-GPU single frame: split rounds sweep (shard_time, every rank on one GPU)
# and the wave timeline of rank 0's recorded-order launch
set -u
OUT=${1:?outdir}; shift; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step rounds 600 python tools/shard_time.py --workload c1 --worlds 1 8 --reps 9 --configs "" RTCLJ_SPLIT_ROUNDS=2 RTCLJ_SPLIT_ROUNDS=4 RTCLJ_SPLIT_ROUNDS=5 "" RTCLJ_SPLIT_ROUNDS=4
grep "N=\|config" $OUT/rounds.log
step tl_r0 200 python tools/timeline.py --workload c1 --world 8 --rank 0 --warm 5 --bins 30 --json $OUT/tl_r0.json
step tl_r7 200 python tools/timeline.py --workload c1 --world 8 --rank 7 --warm 5 --bins 30 --json $OUT/tl_r7.json
step tl_1gpu 200 python tools/timeline.py --workload c1 --world 1 --warm 5 --bins 30 --json $OUT/tl_1gpu.json
echo "== done"
