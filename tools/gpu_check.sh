#!/bin/bash
# One GPU-box pass (run through gpurun from the repo root):
#   tools/gpu_check.sh OUT [stages...]
# stages: tests smoke bench prof pmc dist2 shard (default: all but shard, in that order).
# Every GPU step runs under its own timeout; the first failure ends the pass.
set -u
OUT=${1:?outdir}; shift
STAGES=${*:-"tests smoke bench prof pmc dist2"}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
}
for s in $STAGES; do
  case $s in
    tests) run pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5
           tail -1 "$OUT/bench.log" > "$OUT/bench.json" ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
               python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --e2e off --stats off --pipelined off --sustained 0 ;;
    pmc)   run pmc 900 bash profiles/pmc.sh "$OUT/pmc" ;;
    shard) run shard 300 python tools/shard_time.py --workload c1 --reps 5 --inflight 2 --frames 80
           grep "N=" "$OUT/shard.log" > "$OUT/shard.txt" ;;
    dist2) run dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
               --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3
           tail -1 "$OUT/dist2.log" > "$OUT/dist2.json" ;;
  esac
done
echo "== done"
