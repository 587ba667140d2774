#!/bin/bash
# Round 6 A/B: the record's sort at the next launch (default) against right
# behind the trace kernel (RTCLJ_SORT_EAGER=1), alternated bench runs:
# single frames, bench's pipelined leg, rt_render and rt_render_submit frame
# loops, the first launch of a new shape.   tools/gpu_r6_sort_ab.sh OUT ROUNDS
set -u
OUT=${1:?outdir}; R=${2:-3}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in $(seq 1 "$R"); do
  for S in lazy eager; do
    if [ $S = eager ]; then export RTCLJ_SORT_EAGER=1; else unset RTCLJ_SORT_EAGER; fi
    timeout -k 10 300 python bench.py --cpu-baseline off --stats off --sustained 0 --steps 50 > "$OUT/r${r}_$S.log" 2>&1 || exit $?
    tail -1 "$OUT/r${r}_$S.log" > "$OUT/r${r}_$S.json"
    python -c "
import json; l=json.load(open('$OUT/r${r}_$S.json')); e=l['end_to_end']
print('round $r $S single %.3f pipelined %.3f rt_render %.3f in-flight %.3f first %.3f off %.3f' % (l['single_frame']['ms_per_frame'], l['pipelined']['ms_per_frame'], e['total_ms'], e['frames_in_flight']['ms_per_frame'], l['dispatch_order']['kernel_ms'], l['dispatch_order']['plain_schedule_off_ms']))"
  done
done
unset RTCLJ_SORT_EAGER
