#!/bin/bash
set -u
OUT=gpurun_out/soak; mkdir -p $OUT
for r in 1 2 3; do
  echo "== round $r"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/r$r.log 2>&1
  rc=$?; echo "   rc=$rc"; tail -1 $OUT/r$r.log
  [ $rc -ne 0 ] && exit $rc
done
echo "== done"
