#!/bin/bash
set -u
OUT=gpurun_out/r3n; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 600 python bench.py --steps 20 --warmup 5 --cpu-baseline off
tail -1 $OUT/bench.log > $OUT/bench.json
step e2e 300 python tools/e2e_shards.py --shards 1 8 --reps 5
grep shards= $OUT/e2e.log
echo "== done"
