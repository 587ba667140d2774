#!/bin/bash
# Round 6: the default bench.py line N times back to back on one box (its
# run-to-run spread), one JSON line per run in OUT/bench_reps.jsonl.
set -u
OUT=${1:?outdir}; N=${2:-5}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for i in $(seq 1 "$N"); do
  timeout -k 10 400 python bench.py > "$OUT/bench_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_$i.log" >> "$OUT/bench_reps.jsonl"
  python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[2], round(l['value']), round(l['ms_per_step'], 3), round(l['kernel_ms_avg'], 3), l['end_to_end']['first_process']['process_ms'])" "$OUT/bench_reps.jsonl" "$i"
done
