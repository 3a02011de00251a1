#!/bin/bash
# C2 per-level device times (CRGC_LEVEL_LOG) and a short bench; usage: bash tools/gpu_levels.sh <tag>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-lv}
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 420 python3 "$ROOT/bench.py" --steps 3 --warmup 2 \
  --no-cpu-baseline > "$O/levels.json" 2> "$O/levels.err"
echo levels-done
