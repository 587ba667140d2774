#!/bin/bash
set -u
OUT=gpurun_out/r05d
mkdir -p "$OUT"
export TMPDIR=/tmp
VALU_COST_NEW_ONLY=1 timeout -k 10 120 tools/bin/valu_cost > "$OUT/valu_cost_sgpr.txt" 2>&1; rc=$?; echo "valu_cost rc=$rc"; [ $rc -ne 0 ] && exit $rc
PMC_PASSES="valu1 valu2 waits" bash profiles/pmc.sh "$OUT/pmc_c1" || exit $?
echo done
