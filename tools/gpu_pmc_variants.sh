#!/bin/bash
# PMC insts / waves passes of C1's recorded-order launch per kernel variant
#   tools/gpu_pmc_variants.sh OUT V1 V2 ...
set -u
OUT=${1:?outdir}; shift; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
pmc() { local n=$1 v=$2; shift 2
  step $n 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o prof --pmc "$@" -- \
    python3 tools/launch_frames.py --workload c1 --frames 3 --variant $v
  cp $OUT/$n/prof_counter_collection.csv $OUT/$n.csv; }
for v in "$@"; do
  pmc v${v}_insts $v SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM
  pmc v${v}_waves $v SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
  pmc v${v}_lds $v SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH
  python3 tools/pmc_frames.py $OUT/v${v}_insts.csv $OUT/v${v}_waves.csv $OUT/v${v}_lds.csv > $OUT/v${v}.json
done
echo "== done"
