#!/bin/bash
# Round 6: the rejection-sampler bench line (RT_FLAG_REJECTION_SAMPLERS on
# every launch) and the 8-rank bench rehearsal on the one GPU.
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | grep -v '^{' | tail -3; [ $rc -ne 0 ] && exit $rc; return 0; }
step rejection 400 python bench.py --samplers rejection --e2e off --sustained 0
tail -1 "$OUT/rejection.log" > "$OUT/c1_rejection_samplers.json"
step dist8 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 8 --steps 20 --warmup 3
tail -1 "$OUT/dist8.log" > "$OUT/dist8_rehearsal_one_gpu.json"
echo done
