#!/bin/bash
# round 4: GPU suite, then C1 / C4 HBM bytes of a recorded-order launch (sharing
# off there by default) and C1's steady state with / without sharing in the
# recorded order, first launch per rounds setting
set -u
OUT=${1:?outdir}; shift; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
pmc() { local n=$1 wl=$2 fr=$3; shift 3
  step $n 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o prof --pmc "$@" -- \
    python3 tools/launch_frames.py --workload $wl --frames $fr
  cp $OUT/$n/prof_counter_collection.csv $OUT/$n.csv; }
both() { pmc $1_fetch $2 $3 FETCH_SIZE && pmc $1_write $2 $3 WRITE_SIZE
  python3 tools/pmc_frames.py $OUT/$1_fetch.csv $OUT/$1_write.csv > $OUT/$1_bytes.json; }
both c1 c1 4
both c4 c4 2
step ab_c1 600 python tools/env_ab.py --workload c1 --rounds 4 --reps 10 --set - --set RTCLJ_SHARE_RECORDED=1 --set RTCLJ_SHARE_ROUNDS=3
echo "== done"
