#!/bin/bash
# build_ab.sh REV NAME: the product library built from git revision REV's
# sources, as raytracing-clj_amd/lib/ab_NAME.so (for tools/ab_libs.py)
set -euo pipefail
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
git -C "$ROOT" archive "$REV" raytracing-clj_amd/csrc raytracing-clj_amd/Makefile include | tar -x -C "$T"
make -s -C "$T/raytracing-clj_amd" lib/librtclj.so
cp "$T/raytracing-clj_amd/lib/librtclj.so" "$ROOT/raytracing-clj_amd/lib/ab_$NAME.so"
echo "built raytracing-clj_amd/lib/ab_$NAME.so from $(git -C "$ROOT" rev-parse --short "$REV")"
