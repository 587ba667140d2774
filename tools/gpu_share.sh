#!/bin/bash
# Tile sharing's HBM atomics: PMC bytes per launch of C1 and
# C4 with owners publishing only in the launch's last rounds (default) and
# in every round (RTCLJ_SHARE_ROUNDS=1000000, round 3's rule), plus C1's
# timing A/B of the rule (first launch in plain order, steady state).
#   tools/gpu_share.sh OUT [pytest args...]
set -u
OUT=${1:?outdir}; shift; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
[ $# -gt 0 ] && step tests 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread
pmc() {   # name workload frames counters (env before the call)
  local n=$1 wl=$2 fr=$3; shift 3
  step $n 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o prof --pmc "$@" -- \
    python3 tools/launch_frames.py --workload $wl --frames $fr
  cp $OUT/$n/prof_counter_collection.csv $OUT/$n.csv
}
for wl in c1 c4; do
  fr=4; [ $wl = c4 ] && fr=2
  pmc ${wl}_fetch $wl $fr FETCH_SIZE
  pmc ${wl}_write $wl $fr WRITE_SIZE
  export RTCLJ_SHARE_ROUNDS=1000000
  pmc ${wl}_all_fetch $wl $fr FETCH_SIZE
  pmc ${wl}_all_write $wl $fr WRITE_SIZE
  unset RTCLJ_SHARE_ROUNDS
done
for n in c1 c1_all c4 c4_all; do python3 tools/pmc_frames.py $OUT/${n}_fetch.csv $OUT/${n}_write.csv > $OUT/${n}_bytes.json; done
step ab_c1 600 python tools/env_ab.py --workload c1 --rounds 4 --reps 10 --set - --set RTCLJ_SHARE_ROUNDS=1000000 --set RTCLJ_SHARE_ROUNDS=3 --set RTCLJ_SHARE_ROUNDS=1
echo "== done"
