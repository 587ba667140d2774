#!/bin/bash
# Round 6: the PNG path of a one-frame process on the box's host cores: the
# old and new encoders (tools/bin/png_stages_{old,new}) on C1's scene.ppm,
# alternated, and fresh rt_main processes (png_ms, process_ms).
#   tools/gpu_r6_png.sh OUT
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 60 raytracing-clj_amd/lib/rt_main 100 50 --scene cover --width 1200 --seed 1 --gpus 1 --json \
  --out /tmp/c1.ppm > "$OUT/rt_main_0.json" || exit 1
for i in 1 2 3; do
  timeout -k 10 60 tools/bin/png_stages_old /tmp/c1.ppm /tmp/o.png 9 | sed 's/^/old /' || exit 1
  timeout -k 10 60 tools/bin/png_stages_new /tmp/c1.ppm /tmp/n.png 9 | sed 's/^/new /' || exit 1
done > "$OUT/stages.txt"
cmp /tmp/o.png /tmp/n.png && cmp /tmp/o.png.direct.png /tmp/n.png.direct.png && echo "png bytes identical" >> "$OUT/stages.txt"
ls -l /tmp/c1.ppm /tmp/n.png >> "$OUT/stages.txt"
cp /tmp/c1.ppm "$OUT/c1.ppm"
for i in 1 2 3; do
  timeout -k 10 60 raytracing-clj_amd/lib/rt_main 100 50 --scene cover --width 1200 --seed 1 --gpus 1 --json \
    --out /tmp/c1b.ppm > "$OUT/rt_main_$i.json" || exit 1
done
cat "$OUT/stages.txt"
grep -h -o '"png_ms": [0-9.]*\|"process_ms": [0-9.]*\|"write_ms": [0-9.]*' "$OUT"/rt_main_*.json
