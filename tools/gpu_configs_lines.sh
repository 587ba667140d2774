#!/bin/bash
# BASELINE configs C2-C4 on one MI355X: the bench lines only (tools/gpu_configs.sh adds the shard timings)
set -u
OUT=${1:?outdir}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
B="python bench.py --cpu-baseline off --e2e off"
step c2 400 $B --workload c2
step c3 400 $B --workload c3
step c4 500 $B --workload c4 --steps 2 --warmup 1 --pipelined off
for f in c2 c3 c4; do tail -1 $OUT/$f.log > $OUT/$f.json; done
echo "== done"
