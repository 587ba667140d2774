#!/bin/bash
# Round 6 evidence at the build: PMC passes of C1 and C4 (profiles/pmc.sh),
# the rocprofv3 kernel stats of the C1 bench command, a C1 bench line with
# the statistics leg, and the C2-C4 bench lines.   tools/gpu_r6_pmc.sh OUT [steps]
set -u
OUT=${1:?outdir}; shift
STEPS=${*:-pmc1 prof bench1 configs pmc4}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | grep -v '^{' | tail -4; [ $rc -ne 0 ] && exit $rc; return 0; }
B="python bench.py --cpu-baseline off --e2e off"
for s in $STEPS; do
  case $s in
    pmc1)    step pmc_c1 900 bash profiles/pmc.sh "$OUT/pmc_c1" ;;
    pmc4)    step pmc_c4 1000 bash profiles/pmc.sh "$OUT/pmc_c4" --workload c4 ;;
    prof)    step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- python3 bench.py --cpu-baseline off --e2e off --stats off --pipelined off --sustained 0 --first-launch off ;;
    bench1)  step bench_c1 400 $B --sustained 0; tail -1 "$OUT/bench_c1.log" > "$OUT/c1.json" ;;
    configs) step c2 400 $B --workload c2; tail -1 "$OUT/c2.log" > "$OUT/c2.json"
             step c3 400 $B --workload c3; tail -1 "$OUT/c3.log" > "$OUT/c3.json"
             step c4 500 $B --workload c4 --steps 2 --warmup 1 --pipelined off; tail -1 "$OUT/c4.log" > "$OUT/c4.json" ;;
  esac
done
echo done
