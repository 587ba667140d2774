#!/bin/bash
# One GPU-box pass (run from the repo root via gpurun): GPU parity tests,
# smoke(), the default bench line, and a rocprofv3 kernel-trace/stats pass of
# the same bench command.  Every GPU step has its own time limit; the first
# failing step ends the script.
#   tools/gpu_check.sh <tag> [extra bench.py args]
set -eu
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
echo "pytest ok: $(tail -1 "$OUT/pytest_gpu.log")"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke ok: $(tail -1 "$OUT/smoke.log")"
timeout -k 10 300 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench: $(cat "$OUT/bench.json")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
  python3 bench.py --cpu-baseline off "$@" > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
echo "prof bench: $(cat "$OUT/prof_bench.json")"
