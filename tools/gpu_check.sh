#!/bin/bash
# GPU parity tests, C2 A/B of trace variants with a per-level log, C3 and a
# short C2 bench.  Usage: bash tools/gpu_check.sh <tag> [variant ...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-r1}
shift || true
mkdir -p "$O"
VARS=()
for v in "$@"; do VARS+=(--variant "$v"); done
[ ${#VARS[@]} -eq 0 ] && VARS=(--variant BASE=0)
timeout -k 10 700 python -m pytest tests -m gpu -q -x > "$O/gpu_tests.log" 2>&1 &&
timeout -k 10 400 python tools/ab_trace.py --rounds 6 "${VARS[@]}" > "$O/ab.json" 2> "$O/ab.err" &&
CRGC_LEVEL_LOG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 0 --no-cpu-baseline > "$O/levels.json" 2> "$O/levels.err" &&
timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > "$O/c3.json" 2> "$O/c3.err" &&
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
