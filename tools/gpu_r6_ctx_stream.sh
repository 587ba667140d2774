#!/bin/bash
# Round 6: bench.py's rt_render_submit frame loop (after its pipelined leg has
# used two streams of its own) with the render contexts' streams plain,
# CU-masked or high priority (RTCLJ_CTX_STREAM 0/1/2), alternated.
#   tools/gpu_r6_ctx_stream.sh OUT ROUNDS
set -u
OUT=${1:?outdir}; R=${2:-2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in $(seq 1 "$R"); do
  for K in 0 1 2; do
    RTCLJ_CTX_STREAM=$K timeout -k 10 300 python bench.py --cpu-baseline off --stats off --first-launch off --sustained 0 --steps 50 > "$OUT/r${r}_k$K.log" 2>&1 || exit $?
    tail -1 "$OUT/r${r}_k$K.log" > "$OUT/r${r}_k$K.json"
    python -c "
import json; l=json.load(open('$OUT/r${r}_k$K.json')); e=l['end_to_end']; f=e['frames_in_flight']
print('round $r ctx stream $K: single %.3f rt_render %.3f u8 %.3f in-flight %.3f (last kernel %.3f)' % (l['single_frame']['ms_per_frame'], e['total_ms'], e['bytes']['total_ms'], f['ms_per_frame'], f['kernel_ms_max_last']))"
  done
done
