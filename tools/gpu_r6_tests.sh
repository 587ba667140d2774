#!/bin/bash
# Round 6: variant 28 and the samplers first (a short run), then the whole GPU
# suite, smoke, the per-rank shard timings of C1 with and without 28, and a
# default bench line.   tools/gpu_r6_tests.sh OUT
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "28 or compact or mirror_fixture or scene_matches" > "$OUT/quick.log" 2>&1
rc=$?; echo "quick rc=$rc"; tail -3 "$OUT/quick.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/shard_time.py --workload c1 --worlds 1 2 4 8 --reps 9 --configs "" "RTCLJ_TH4=0" > "$OUT/shard_c1.txt" 2>&1
rc=$?; echo "shard rc=$rc"; tail -12 "$OUT/shard_c1.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
echo done
