#!/bin/bash
# C4 A/B of two library builds: the variant-18 parity tests through each,
# then C4 bench lines alternated.  tools/gpu_r5c4.sh OUT libA libB
set -u
OUT=$1; A=$2; B=$3; mkdir -p "$OUT"; export TMPDIR=/tmp
for L in "$A" "$B"; do
  n=$(basename "$L" .so)
  RTCLJ_LIBRARY=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "18 or c4" -q --timeout 200 --timeout-method thread > "$OUT/tests_$n.log" 2>&1 || { tail -20 "$OUT/tests_$n.log"; exit 1; }
  tail -1 "$OUT/tests_$n.log"
done
for r in 1 2; do
  for L in "$A" "$B"; do
    n=$(basename "$L" .so)
    RTCLJ_LIBRARY=$PWD/$L timeout -k 10 300 python bench.py --cpu-baseline off --e2e off --stats off --workload c4 --steps 2 --warmup 1 --pipelined off --sustained 0 > "$OUT/c4_${n}_$r.log" 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('$OUT/c4_${n}_$r.log').read().strip().splitlines()[-1]); print('$n', $r, round(d['value']), round(d['kernel_ms_avg'],1))"
  done
done
