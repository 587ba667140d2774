#!/bin/bash
# PMC recipe (MI355X_MICROARCH.md §rocprofv3 / §HBM): one counter group per
# rocprofv3 pass, kernel-trace + stats only (no sys/runtime traces), on the
# bench's own command.  Usage (on the GPU box, from the repo root):
#   profiles/pmc.sh gpurun_out/pmc [extra bench.py args]
# Writes <out>/<pass>/prof_counter_collection.csv per pass, copied to
# <out>/<pass>.csv (the form committed under profiles/rNN/ and read by bench.py).
set -u
OUT=${1:?outdir}; shift
REPO=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$REPO" || exit 1
mkdir -p "$OUT"
BENCH=(python3 bench.py --cpu-baseline off --e2e off --stats off --pipelined off --sustained 0 --first-launch off --steps 2 --warmup 1 "$@")
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o prof \
    --pmc "$@" -- "${BENCH[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  [ -f "$OUT/$name/prof_counter_collection.csv" ] && cp "$OUT/$name/prof_counter_collection.csv" "$OUT/$name.csv"
  case $rc in 124|134|137|139) echo "stopping: GPU step failed ($rc)"; exit $rc ;; esac
  return 0
}
PASSES=${PMC_PASSES:-"valu1 valu2 waits fetch write"}
for g in $PASSES; do
  case $g in
    waves) pass waves SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE ;;
    insts) pass insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU ;;
    lds)   pass lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH ;;
    sched) pass sched SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES ;;
    valu1) pass valu1 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE ;;
    valu2) pass valu2 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE ;;
    waits) pass waits SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE ;;
    fetch) pass fetch FETCH_SIZE ;;
    write) pass write WRITE_SIZE ;;
  esac
done
