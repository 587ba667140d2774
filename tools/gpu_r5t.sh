#!/bin/bash
# GPU suite + smoke + C1 bench line + C2/C3/C4 lines at the current build.
#   tools/gpu_r5t.sh OUT [configs]   (configs: "c2 c3 c4", default c2)
set -u
OUT=${1:?outdir}; CFG=${2:-c2}
bash tools/gpu_tests.sh "$OUT" || exit $?
export TMPDIR=/tmp
for c in $CFG; do
  extra=""; [ "$c" = "c4" ] && extra="--steps 2 --warmup 1 --pipelined off"
  timeout -k 10 500 python bench.py --cpu-baseline off --e2e off --workload $c $extra > "$OUT/$c.log" 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/$c.log"; exit $rc; }
  tail -1 "$OUT/$c.log" > "$OUT/$c.json"
done
echo all-done
