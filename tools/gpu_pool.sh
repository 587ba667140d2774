#!/bin/bash
set -u
OUT=${1:?outdir}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -40 $OUT/$n.log; exit $rc; fi; }
L=$PWD/raytracing-clj_amd/lib
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_host_paths.py tests/test_jni_shim.py -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
  step new$r 120 python tools/fanout_overhead.py
  step old$r 120 env RTCLJ_LIBRARY=$L/ab_r3.so python tools/fanout_overhead.py
done
tail -n1 $OUT/new*.log $OUT/old*.log
echo "== done"
