#!/bin/bash
set -u
OUT=gpurun_out/r3c; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step head 200 env RTCLJ_LIBRARY=raytracing-clj_amd/lib/ab_head.so python tools/shard_time.py --workload c1 --reps 5 --worlds 1 8
step cur 400 python tools/shard_time.py --workload c1 --reps 5 --worlds 1 8 --configs "RTCLJ_STEAL=0,RTCLJ_PERSIST=0" "RTCLJ_STEAL=0" "RTCLJ_PERSIST=0" ""
grep -h "N=\|config" $OUT/head.log $OUT/cur.log
echo "== done"
