#!/bin/bash
# Round 6: one-frame processes (rt_main, C1) alternated between two builds
# (tools/bin/old, tools/bin/new: rt_main + librtclj.so side by side), for the
# start-up's parts; OUT/ab.jsonl one line per process.
set -u
OUT=${1:?outdir}; N=${2:-6}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" || exit 1
for i in $(seq 1 "$N"); do
  for b in old new; do
    timeout -k 10 60 tools/bin/$b/rt_main 100 50 --scene cover --width 1200 --seed 1 --gpus 1 --json \
      --out /tmp/ab_$b.ppm > "$OUT/$b.$i.log" 2>&1 || exit 1
    echo "{\"build\": \"$b\", \"run\": $i, \"line\": $(tail -1 "$OUT/$b.$i.log")}" >> "$OUT/ab.jsonl"
  done
done
cmp /tmp/ab_old.ppm /tmp/ab_new.ppm && echo "ppm identical"
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, statistics as S
rows = [json.loads(l) for l in open(sys.argv[1])]
for b in ("old", "new"):
    r = [x["line"] for x in rows if x["build"] == b]
    f = lambda k: [round(x[k], 1) for x in r]
    print(b, "process", f("process_ms"), "median", round(S.median(x["process_ms"] for x in r), 1))
    print(b, "  prepare_wait", f("prepare_wait_ms"), "device_count", f("device_count_ms"))
    print(b, "  parts", [[round(v, 1) for v in x["prepare_ms"].values()] for x in r])
    print(b, "  render", f("render_ms"), "png", f("png_ms"))
PY
