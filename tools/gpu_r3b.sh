#!/bin/bash
# round-3 stealing check: steal tests first, then the suite, then timings
set -u
OUT=gpurun_out/r3b; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step steal 240 python -u -m pytest tests/test_gpu_steal.py -x -v --timeout 120 --timeout-method thread
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench1 300 python bench.py --steps 20 --warmup 5 --inflight 1 --cpu-baseline off
tail -1 $OUT/bench1.log > $OUT/bench1.json
step shard 300 python tools/shard_time.py --workload c1 --reps 5
step shard_nosteal 300 env RTCLJ_STEAL=0 python tools/shard_time.py --workload c1 --reps 5
echo "== done"
