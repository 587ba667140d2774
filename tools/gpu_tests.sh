#!/bin/bash
# GPU test suite + smoke + a default bench line at the current build.
#   tools/gpu_tests.sh OUT
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
echo done
