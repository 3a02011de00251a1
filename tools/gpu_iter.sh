#!/bin/bash
# One build -> measure iteration: GPU parity suite, per-level log with every level
# kernel timed, interleaved A/B of trace variants (env switches).
# usage: bash tools/gpu_iter.sh <tag> [variant ...]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-iter}
mkdir -p "$O"
shift || true
cd "$ROOT"
VARS=()
for v in "$@"; do VARS+=(--variant "$v"); done
[ ${#VARS[@]} -eq 0 ] && VARS=(--variant BASE=0)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$O/gpu_tests.log" 2>&1
CRGC_KERNEL_TIMING=2 CRGC_LEVEL_LOG=1 timeout -k 10 300 python tools/ab_trace.py --rounds 1 --variant BASE=0 \
  > "$O/levels.json" 2> "$O/levels.err"
timeout -k 10 400 python tools/ab_trace.py --rounds 6 "${VARS[@]}" > "$O/ab.json" 2> "$O/ab.err"
echo iter-done
