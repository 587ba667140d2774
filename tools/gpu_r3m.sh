#!/bin/bash
set -u
OUT=gpurun_out/r3m; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step first_call 60 tools/first_call
cat $OUT/first_call.log
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 600 python bench.py --steps 20 --warmup 5
tail -1 $OUT/bench.log > $OUT/bench.json
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --e2e off --stats off
echo "== done"
