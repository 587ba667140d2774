#!/bin/bash
# Round 6: rt_render_submit's frame loop inside bench.py with the legs before
# it switched off one at a time (which earlier leg leaves it at ~4.96 ms per
# C1 frame against 4.69 in a fresh process).   tools/gpu_r6_inflight_legs.sh OUT
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
i=0
for r in 1 2; do
  for LEGS in "" "--first-launch off" "--pipelined off" "--first-launch off --pipelined off" "--first-launch off --pipelined off --stats off"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --cpu-baseline off --sustained 0 --steps 50 $LEGS > "$OUT/run$i.log" 2>&1 || exit $?
    tail -1 "$OUT/run$i.log" > "$OUT/run$i.json"
    python -c "
import json; l=json.load(open('$OUT/run$i.json')); e=l['end_to_end']; f=e['frames_in_flight']
print('run $i [$LEGS]: rt_render %.3f in-flight %.3f (last kernel %.3f)' % (e['total_ms'], f['ms_per_frame'], f['kernel_ms_max_last']))"
  done
done
