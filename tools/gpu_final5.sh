#!/bin/bash
# Round-5 validation and evidence on one MI355X (run through gpurun from the repo root):
#   tools/gpu_final5.sh OUT [steps...]   (default: every step, in this order)
# GPU tests, smoke, PMC passes of C1 and C4 (copied to profiles/r05/pmc_*, which the
# bench line reads), the default bench line (with its CPU baseline), its rocprofv3
# summary, the 2- and 8-rank rehearsals (8 ranks share this one GPU; the product
# fan-out's 8 shards go to device 0) and the C1 shard timings.
set -u
OUT=${1:?outdir}; shift; mkdir -p $OUT; export TMPDIR=/tmp
STEPS=${*:-"tests smoke pmc_c1 pmc_c4 bench prof dist2 dist8 shard"}
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
for s in $STEPS; do
  case $s in
    tests) step tests 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    smoke) step smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pmc_c1) step pmc_c1 900 bash profiles/pmc.sh $OUT/pmc_c1 --steps 6 --warmup 2
            mkdir -p profiles/r05/pmc_c1 && cp $OUT/pmc_c1/*.csv profiles/r05/pmc_c1/ ;;
    pmc_c4) step pmc_c4 1000 bash profiles/pmc.sh $OUT/pmc_c4 --workload c4 --steps 2 --warmup 0
            mkdir -p profiles/r05/pmc_c4 && cp $OUT/pmc_c4/*.csv profiles/r05/pmc_c4/ ;;
    bench) step bench 600 python bench.py; tail -1 $OUT/bench.log > $OUT/bench.json ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --cpu-baseline off --e2e off --stats off --pipelined off --sustained 0 ;;
    dist2) step dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-baseline off
           tail -1 $OUT/dist2.log > $OUT/dist2.json ;;
    dist8) step dist8 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --steps 10 --warmup 3 --cpu-baseline off
           tail -1 $OUT/dist8.log > $OUT/dist8.json ;;
    configs) for c in c2 c3 c4; do
               extra=""; [ "$c" = "c4" ] && extra="--steps 2 --warmup 1 --pipelined off"
               step $c 500 python bench.py --cpu-baseline off --e2e off --workload $c $extra
               tail -1 $OUT/$c.log > $OUT/$c.json
             done ;;
    shard) step shard 400 python tools/shard_time.py --workload c1 --reps 9 --inflight 2 --frames 80
           grep "N=" $OUT/shard.log ;;
  esac
done
echo "== done"
