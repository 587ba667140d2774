#!/bin/bash
set -u
OUT=gpurun_out/r3i; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step steal 240 python -u -m pytest tests/test_gpu_steal.py -x -v --timeout 120 --timeout-method thread
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 5
tail -1 $OUT/bench.log > $OUT/bench.json
step bench1 300 python bench.py --steps 20 --warmup 5 --inflight 1 --cpu-baseline off
tail -1 $OUT/bench1.log > $OUT/bench1.json
step shard 300 python tools/shard_time.py --workload c1 --reps 5 --inflight 2 --frames 80
grep "N=" $OUT/shard.log
echo "== done"
