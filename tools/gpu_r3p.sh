#!/bin/bash
set -u
OUT=gpurun_out/r3p; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
L=raytracing-clj_amd/lib
step steal 240 python -u -m pytest tests/test_gpu_steal.py -x -q --timeout 120 --timeout-method thread
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step head 200 env RTCLJ_LIBRARY=$L/ab_head.so python tools/shard_time.py --workload c1 --reps 7 --worlds 1 8
step cur 400 python tools/shard_time.py --workload c1 --reps 7 --worlds 1 8 --configs "" "RTCLJ_STEAL=0" "RTCLJ_SPLIT=1"
grep -h "N=\|config" $OUT/head.log $OUT/cur.log
step bench1 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off
tail -1 $OUT/bench1.log > $OUT/bench1.json
echo "== done"
