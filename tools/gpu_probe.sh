#!/bin/bash
# cost probe for a shape's first launch: tests, bench new-shape time with the probe on / off, timelines
set -u
OUT=${1:-gpurun_out/probe}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
B="python bench.py --cpu-baseline off --e2e off --stats off --steps 20 --warmup 3"
step tests 300 python -u -m pytest tests/test_gpu_schedule.py -x -q --timeout 120 --timeout-method thread
step on1 300 $B
step off1 300 env RTCLJ_PROBE=0 $B
step on2 300 $B
step off2 300 env RTCLJ_PROBE=0 $B
step c4_on 600 python bench.py --cpu-baseline off --e2e off --stats off --workload c4 --steps 1 --warmup 1
for f in on1 off1 on2 off2 c4_on; do tail -1 $OUT/$f.log > $OUT/$f.json; done
step tl_probe 200 python tools/timeline.py --workload c1 --world 1 --warm 0 --bins 30
echo "== done"
