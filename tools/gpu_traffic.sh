#!/bin/bash
# C1 HBM bytes per launch (PMC FETCH_SIZE / WRITE_SIZE) with tile sharing on / off, compaction on / off
set -u
OUT=${1:-gpurun_out/traffic}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step def 300 env PMC_PASSES="fetch write" bash profiles/pmc.sh $OUT/def --steps 4 --warmup 2
step nosteal 300 env RTCLJ_STEAL=0 PMC_PASSES="fetch write" bash profiles/pmc.sh $OUT/nosteal --steps 4 --warmup 2
step nocompact 300 env RTCLJ_COMPACT=0 PMC_PASSES="fetch write" bash profiles/pmc.sh $OUT/nocompact --steps 4 --warmup 2
echo "== done"
