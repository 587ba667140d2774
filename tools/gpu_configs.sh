#!/bin/bash
# BASELINE configs C2-C4 on one MI355X: bench lines and the C3/C4 8-rank shard timings
set -u
OUT=${1:?outdir}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
B="python bench.py --cpu-baseline off --e2e off"
step c2 600 $B --workload c2
step c3 600 $B --workload c3
step c4 900 $B --workload c4 --steps 2 --warmup 1 --pipelined off
for f in c2 c3 c4; do tail -1 $OUT/$f.log > $OUT/$f.json; done
step shard_c3 600 python tools/shard_time.py --workload c3 --reps 3 --worlds 1 8
step shard_c4 900 python tools/shard_time.py --workload c4 --reps 2 --worlds 1 8
grep "N=" $OUT/shard_c3.log $OUT/shard_c4.log
echo "== done"
