#!/bin/bash
# Round-6 A/B of the loop-free samplers (RTCLJ_SAMPLER bits: 1 sphere, 2 disk)
# on C1, alternated per round with the HEAD build (ab_base.so):
#   tools/gpu_r6_sampler.sh OUT ROUNDS [settings...]   (settings: base 0 1 2 3)
# then one parity run (bench.py's CPU leg: REF64 rows vs the GPU frame) with
# both samplers on.  Every run has its own time limit; the first failure ends it.
set -u
OUT=$1; ROUNDS=$2; shift 2
SETS=${*:-base 0 1 3}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 "$ROUNDS"); do
  for S in $SETS; do
    if [ "$S" = base ]; then L=raytracing-clj_amd/lib/ab_base.so; SS=0; else L=raytracing-clj_amd/lib/librtclj.so; SS=$S; fi
    RTCLJ_LIBRARY=$PWD/$L RTCLJ_SAMPLER=$SS timeout -k 10 240 python bench.py --cpu-baseline off --e2e off \
      --sustained 0 --pipelined off --steps 30 --warmup 3 > "$OUT/r${r}_$S.json" 2> "$OUT/r${r}_$S.err" || exit $?
    python -c "import json; l=json.loads(open('$OUT/r${r}_$S.json').read().strip().splitlines()[-1]); \
print('round $r sampler $S kernel', l['kernel_ms_avg'], 'value', round(l['value']), 'plain', (l.get('dispatch_order') or {}).get('kernel_ms'))"
  done
done
if [ -n "${PARITY:-}" ]; then
  RTCLJ_SAMPLER=$PARITY timeout -k 10 300 python bench.py --e2e off --sustained 0 --pipelined off --steps 20 \
    --warmup 3 > "$OUT/parity_$PARITY.json" 2> "$OUT/parity_$PARITY.err" || exit $?
  python -c "import json; l=json.loads(open('$OUT/parity_$PARITY.json').read().strip().splitlines()[-1]); print('parity', json.dumps(l.get('parity')))"
fi
