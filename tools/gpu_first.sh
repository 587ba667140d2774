#!/bin/bash
# first launch of a new shape vs the schedule off, after warm-up: C1 bench x3, C4 once
set -u
OUT=${1:-gpurun_out/first}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
B="python bench.py --cpu-baseline off --e2e off --stats off --pipelined off --sustained 0 --steps 20 --warmup 3"
step b1 300 $B
step b2 300 $B
step b3 300 $B
for f in b1 b2 b3; do tail -1 $OUT/$f.log > $OUT/$f.json; done
echo "== done"
