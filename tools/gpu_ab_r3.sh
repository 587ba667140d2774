#!/bin/bash
# round-3 build (lib/ab_r3.so) vs the working build on C2 and C1, alternated
set -u
OUT=${1:?outdir}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
L=$PWD/raytracing-clj_amd/lib
step ab_c2 900 python tools/ab_libs.py --libs $L/ab_r3.so $L/librtclj.so --rounds 3 --steps 6 -- --workload c2 --stats off --e2e off --pipelined off --sustained 0
step ab_c1 600 python tools/ab_libs.py --libs $L/ab_r3.so $L/librtclj.so --rounds 3 --steps 40 -- --stats off --e2e off --pipelined off --sustained 0
tail -4 $OUT/ab_c2.log; tail -4 $OUT/ab_c1.log
echo "== done"
