#!/bin/bash
# Round 6: the GPU suite, smoke, a default bench line, and the per-rank shard
# timings of C1 (single frame, 2 frames in flight), C3 and C4 at the build.
#   tools/gpu_r6_suite.sh OUT [steps...]   (steps: tests smoke bench shard1 shard34; default all)
set -u
OUT=${1:?outdir}; shift
STEPS=${*:-tests smoke bench shard1 shard34}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | grep -v '^\[{' | tail -12; [ $rc -ne 0 ] && exit $rc; return 0; }
for s in $STEPS; do
  case $s in
    tests)   step pytest 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke)   step smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   step bench 400 python bench.py; tail -1 "$OUT/bench.log" > "$OUT/bench.json" ;;
    shard1)  step shard_c1 400 python -u tools/shard_time.py --workload c1 --worlds 1 2 4 8 --reps 9 --inflight 2 --frames 40 ;;
    shard34) step shard_c3 600 python -u tools/shard_time.py --workload c3 --worlds 1 8 --reps 3
             step shard_c4 900 python -u tools/shard_time.py --workload c4 --worlds 1 8 --reps 2 ;;
  esac
done
echo done
