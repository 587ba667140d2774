#!/bin/bash
# Round 5: VALU cost table (more opcodes) + PMC passes of the VALU mix on C1.
set -u
OUT=gpurun_out/r05b
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 tools/bin/valu_cost > "$OUT/valu_cost.txt" 2>&1; rc=$?; echo "valu_cost rc=$rc"; [ $rc -ne 0 ] && exit $rc
PMC_PASSES="valu1 valu2 waits" bash profiles/pmc.sh "$OUT/pmc_c1" || exit $?
echo done
