#!/bin/bash
# A/B of a kernel change on one MI355X (through gpurun, from the repo root):
#   tools/build_ab.sh HEAD head        # (here, before the call) the base build
#   tools/gpu_ab.sh OUT [TESTS...]     # on the box
# the given GPU tests, then alternating bench runs of ab_head.so and the working
# build (tools/ab_libs.py) and the PMC instruction pass of each
set -u
OUT=${1:?outdir}; shift; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
L=$PWD/raytracing-clj_amd/lib
[ $# -gt 0 ] && step tests 600 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread
step ab 600 python tools/ab_libs.py --libs $L/ab_head.so $L/librtclj.so --rounds 3 --steps 30 -- --stats off --e2e off --pipelined off --sustained 0
step pmc_head 300 env RTCLJ_LIBRARY=$L/ab_head.so PMC_PASSES="insts" bash profiles/pmc.sh $OUT/pmc_head --steps 2 --warmup 1
step pmc_new 300 env PMC_PASSES="insts" bash profiles/pmc.sh $OUT/pmc_new --steps 2 --warmup 1
echo "== done"
