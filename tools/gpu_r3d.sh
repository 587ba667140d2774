#!/bin/bash
set -u
OUT=gpurun_out/r3d; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
L=raytracing-clj_amd/lib
for lib in ab_head librtclj ab_B1 ab_B2 ab_B3 ab_head librtclj; do
  step $lib 200 env RTCLJ_LIBRARY=$L/$lib.so python tools/shard_time.py --workload c1 --reps 7 --worlds 1 --configs "RTCLJ_STEAL=0,RTCLJ_PERSIST=0" "RTCLJ_STEAL=0"
  grep -h "N=\|config" $OUT/$lib.log
done
echo "== done"
