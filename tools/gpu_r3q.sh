#!/bin/bash
# round-3 profiles of the sharing build: PMC passes (C1, C4), bench lines of C2-C4, C3/C4 shard timings
set -u
OUT=gpurun_out/r3q; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step pmc_c1 900 bash profiles/pmc.sh $OUT/pmc_c1
for w in c2 c3 c4; do
  step bench_$w 600 python bench.py --workload $w --cpu-baseline off
  tail -1 $OUT/bench_$w.log > $OUT/bench_$w.json
done
step shard_c3 600 python tools/shard_time.py --workload c3 --reps 3 --worlds 1 8
step shard_c4 900 python tools/shard_time.py --workload c4 --reps 2 --worlds 1 8
grep -h "N=" $OUT/shard_c3.log $OUT/shard_c4.log
step pmc_c4 900 env PMC_PASSES="waves insts fetch write" bash profiles/pmc.sh $OUT/pmc_c4 --workload c4 --steps 1 --warmup 0
echo "== done"
