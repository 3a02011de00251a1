#!/bin/bash
# Per-level log of a C2 trace and an interleaved A/B of trace variants.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-r1}
mkdir -p "$O"
shift || true
VARS=()
for v in "$@"; do VARS+=(--variant "$v"); done
[ ${#VARS[@]} -eq 0 ] && VARS=(--variant BASE=0)
CRGC_LEVEL_LOG=1 timeout -k 10 300 python tools/ab_trace.py --rounds 1 --variant BASE=0 > "$O/levels.json" 2> "$O/levels.err"
timeout -k 10 400 python tools/ab_trace.py --rounds 6 "${VARS[@]}" > "$O/ab.json" 2> "$O/ab.err"
echo levels-done
