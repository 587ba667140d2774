#!/bin/bash
# One-frame-per-process C1 (rt_main, cover 1200x675 100 spp): the frame
# quantised on the device (rt_render_u8, default) against rt_render's floats
# + rt_quantize on the host (--host-quantize), alternated; one JSON per run.
set -u
OUT=${1:?outdir}; REPS=${2:-4}; mkdir -p $OUT
EXE=raytracing-clj_amd/lib/rt_main
for i in $(seq 1 $REPS); do
  for mode in device host; do
    extra=""; [ $mode = host ] && extra="--host-quantize"
    timeout -k 10 120 $EXE 100 50 --scene cover --width 1200 --seed 1 --gpus 1 --out /tmp/fp_$mode.ppm --json $extra > $OUT/run.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then cat $OUT/run.log; exit $rc; fi
    tail -1 $OUT/run.log >> $OUT/first_process_$mode.jsonl
  done
done
cmp /tmp/fp_device.ppm /tmp/fp_host.ppm && echo "ppm identical"
