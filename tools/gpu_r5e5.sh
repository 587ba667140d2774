#!/bin/bash
# A/B of two library builds on C1 (tools/gpu_ab5.sh), then the HBM PMC
# passes of the second:  tools/gpu_r5e5.sh OUT libA libB
set -u
OUT=$1; A=$2; B=$3
bash tools/gpu_ab5.sh "$OUT" 4 "$A" "$B" ${EXTRA_LIBS:-} || exit $?
export RTCLJ_LIBRARY=$PWD/$B
PMC_PASSES="fetch write" timeout -k 10 300 bash profiles/pmc.sh "$OUT/pmc_b" --steps 6 --warmup 2 || exit $?
python3 tools/pmc_summary.py "$OUT/pmc_b" | tail -3
