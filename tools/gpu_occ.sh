#!/bin/bash
# Occupancy sensitivity of the default kernel (diagnostic build): C1 bench
# runs with RTCLJ_LDS_PAD extra dynamic LDS per workgroup -- 0 (6 per CU),
# 4096 (5), 12288 (4) -- alternated over rounds, one process each.
#   tools/gpu_occ.sh OUT [ROUNDS]
set -u
OUT=${1:?outdir}; R=${2:-2}; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/raytracing-clj_amd/lib/librtclj_diag.so
for r in $(seq 1 $R); do
  for pad in 0 4096 12288; do
    RTCLJ_LIBRARY=$L RTCLJ_LDS_PAD=$pad timeout -k 10 240 python bench.py --cpu-baseline off --e2e off --stats off \
      --pipelined off --sustained 0 --steps 30 --warmup 3 > $OUT/occ_${pad}_$r.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "pad $pad rc=$rc"; tail -20 $OUT/occ_${pad}_$r.log; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open('$OUT/occ_${pad}_$r.log').read().strip().splitlines()[-1]); print('round $r pad $pad', round(d['kernel_ms_avg'],3), 'ms', d.get('occupancy'))"
  done
done
