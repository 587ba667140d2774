#!/bin/bash
# Round-end validation and evidence on one MI355X (run through gpurun from the repo root):
#   tools/gpu_final.sh OUT
# GPU tests, smoke, the default bench line (with its CPU baseline), its rocprofv3
# summary, PMC passes of C1 and C4, the 2-rank rehearsal and the C1 shard timings.
set -u
OUT=${1:?outdir}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
step pmc_c1 900 bash profiles/pmc.sh $OUT/pmc_c1 --steps 6 --warmup 2
step pmc_c4 900 env PMC_PASSES="waves insts fetch write" bash profiles/pmc.sh $OUT/pmc_c4 --workload c4 --steps 3 --warmup 1
# the bench line reads its PMC fields from profiles/r04/pmc_{c1,c4}: this build's passes
# (copy them there in the repo too, after the call)
mkdir -p profiles/r04/pmc_c1 profiles/r04/pmc_c4; for w in c1 c4; do cp $OUT/pmc_$w/*.csv profiles/r04/pmc_$w/; done
step bench 600 python bench.py
tail -1 $OUT/bench.log > $OUT/bench.json
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --cpu-baseline off --e2e off --stats off --pipelined off --sustained 0
step dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-baseline off
tail -1 $OUT/dist2.log > $OUT/dist2.json
step dist4 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 10 --warmup 3 --cpu-baseline off
tail -1 $OUT/dist4.log > $OUT/dist4.json
step shard 300 python tools/shard_time.py --workload c1 --reps 9 --inflight 2 --frames 80
grep "N=" $OUT/shard.log
echo "== done"
