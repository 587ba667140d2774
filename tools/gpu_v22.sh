#!/bin/bash
# A/B: a base build's default against a new build's default and its variant
# 22 (seven workgroups per CU), C1 bench runs alternated, one process each.
#   tools/gpu_v22.sh OUT BASE.so NEW.so [ROUNDS]
set -u
OUT=${1:?outdir}; BASE=${2:?base lib}; NEW=${3:?new lib}; R=${4:-3}; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # name lib variant
  RTCLJ_LIBRARY=$2 timeout -k 10 240 python bench.py --cpu-baseline off --e2e off --stats off --pipelined off \
    --sustained 0 --steps 30 --warmup 3 --variant $3 > $OUT/$1_$r.log 2>&1
  local rc=$?; if [ $rc -ne 0 ]; then echo "$1 rc=$rc"; tail -20 $OUT/$1_$r.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('$OUT/$1_$r.log').read().strip().splitlines()[-1]); o=d.get('occupancy',{}); print('round $r $1', round(d['kernel_ms_avg'],3), 'ms plain', round((d.get('dispatch_order') or {}).get('kernel_ms',0),3), 'variant', o.get('variant'), 'wg/cu', o.get('workgroups_per_cu'), 'vgprs', o.get('vgprs'))"
}
for r in $(seq 1 $R); do
  run base $BASE 0
  run new16 $NEW 0
  run new22 $NEW 22
done
