#!/bin/bash
# GPU suite, C1 shard timings with cost-balanced splits on / off, the bench line
set -u
OUT=${1:?outdir}; shift; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step shard 600 python tools/shard_time.py --workload c1 --reps 9 --configs "" "RTCLJ_SPLIT_PLAN=0" "" "RTCLJ_SPLIT_PLAN=0"
grep "N=\|config" $OUT/shard.log
step bench 600 python bench.py
tail -1 $OUT/bench.log > $OUT/bench.json
echo "== done"
