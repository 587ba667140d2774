#!/bin/bash
# C1 knob sweep (env_ab: plain-order first launch + recorded-order steady state, same box)
set -u
OUT=${1:?outdir}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step batch 900 python tools/env_ab.py --workload c1 --rounds 6 --warm 3 --reps 20 --set - --set RTCLJ_LDS_BATCH=128 --set RTCLJ_LDS_BATCH=512 --set RTCLJ_LDS_BATCH=384
step compact 900 python tools/env_ab.py --workload c1 --rounds 6 --warm 3 --reps 20 --set - --set RTCLJ_COMPACT=16 --set RTCLJ_COMPACT=10 --set RTCLJ_COMPACT=0
echo "== done"
