#!/bin/bash
# direction-coherent waves (variants 20/21) vs the default traversal (16):
# parity tests, then an interleaved timing A/B on C1 (recorded order)
set -u
OUT=${1:?outdir}; shift; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
[ "${SKIP_TESTS:-0}" = 1 ] || step tests 600 python -u -m pytest tests/test_gpu_sorted.py -m gpu -x -v --timeout 300 --timeout-method thread
step ab 600 python tools/ab.py --persistent --variants 16 20 21 --rounds 3
tail -8 $OUT/ab.log
echo "== done"
