#!/bin/bash
# Round 6: the first frame's parts (host rt_launch calls, rocprof kernel
# durations of a fresh process's first launches and of the schedule on/off
# alternation) and variant 28's per-sample cost on the whole C1 frame.
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -6; [ $rc -ne 0 ] && exit $rc; return 0; }
step cold 300 python -u tools/first_frame.py --workload c1 --rounds 9 --cold --json "$OUT/first_frame.json"
step prof_cold 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cold" -o prof -- python3 tools/first_frame.py --child 0 0
step prof_alt 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_alt" -o prof -- python3 tools/first_frame.py --rounds 5
for v in 22 28 22 28; do
  step bench_v$v 300 python bench.py --variant $v --cpu-baseline off --e2e off --sustained 0 --pipelined off --stats off --steps 20 --warmup 3
  tail -1 "$OUT/bench_v$v.log" >> "$OUT/bench_v$v.jsonl"
done
echo done
