#!/bin/bash
# Round 6's evidence at the final build: the GPU suite, smoke, the default
# bench line, its rocprofv3 kernel summary (timed frames only), and the 2-rank
# bench rehearsal on the one GPU.   tools/gpu_r6_final.sh OUT [steps]
set -u
OUT=${1:?outdir}; shift
STEPS=${*:-tests smoke bench prof dist2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | grep -v '^{' | tail -3; [ $rc -ne 0 ] && exit $rc; return 0; }
for s in $STEPS; do
  case $s in
    tests) step pytest 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke) step smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 400 python bench.py; tail -1 "$OUT/bench.log" > "$OUT/c1_bench.json" ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- python3 bench.py --cpu-baseline off --e2e off --stats off --pipelined off --sustained 0 --first-launch off ;;
    dist2) step dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 3
           tail -1 "$OUT/dist2.log" > "$OUT/dist2_rehearsal_one_gpu.json" ;;
  esac
done
echo done
