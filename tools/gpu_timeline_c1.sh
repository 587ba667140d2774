#!/bin/bash
set -u
OUT=gpurun_out/tl; mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -20 $OUT/$n.log; exit $rc; fi; }
step plain 200 python tools/timeline.py --workload c1 --world 1 --warm 0 --bins 30
step recorded 200 python tools/timeline.py --workload c1 --world 1 --warm 3 --bins 30
step plain_nosteal 200 env RTCLJ_STEAL=0 python tools/timeline.py --workload c1 --world 1 --warm 0 --bins 30
echo "== done"
