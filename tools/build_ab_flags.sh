#!/bin/bash
# build_ab_flags.sh NAME [extra hipcc flags...]: the product library from the
# working tree's sources with extra compile flags (A/B switches such as
# -DRTCLJ_UNPACK=1), as raytracing-clj_amd/lib/ab_NAME.so (tools/ab_libs.py);
# variant 26's kernel is linked from the Makefile's lib/trace_w16.o as built
# (the Makefile's flags; a later -mllvm -amdgpu-sched-strategy=... overrides)
set -euo pipefail
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
P=$ROOT/raytracing-clj_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -fvisibility=hidden \
  -fvisibility-inlines-hidden -mllvm -vectorize-slp=false -mllvm -amdgpu-sched-strategy=max-ilp "$@" -shared -o "$P/lib/ab_$NAME.so" \
  $P/csrc/trace.hip $P/csrc/rt_host.cpp $P/csrc/scenes.cpp $P/csrc/bvh.cpp $P/csrc/png.cpp \
  -x none $P/lib/trace_w16.o -lz 2>&1 | grep -v "hip-link" || true
test -f "$P/lib/ab_$NAME.so" && echo "built lib/ab_$NAME.so ($*)"
