#!/bin/bash
# guided claims from the workgroup's LDS counter (RTCLJ_LDS_BATCH: 64 = round 3's fixed batches)
set -u
OUT=${1:?outdir}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step tests 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread
step c2 900 python tools/env_ab.py --workload c2 --rounds 3 --warm 2 --reps 5 --set - --set RTCLJ_LDS_BATCH=256 --set RTCLJ_LDS_BATCH=1024
step c1 900 python tools/env_ab.py --workload c1 --rounds 4 --warm 3 --reps 20 --set - --set RTCLJ_LDS_BATCH=256 --set RTCLJ_LDS_BATCH=1024
tail -1 $OUT/c2.log; tail -1 $OUT/c1.log
echo "== done"
