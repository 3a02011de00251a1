#!/bin/bash
# A diagnostic build's C2 bench (its device printf lines land in the .out file):
#   bash tools/gpu_diag.sh <tag> <lib.so>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
mkdir -p "$O"
cd /tmp
CRGC_LIB_AB=$ROOT/$2 timeout -k 10 300 python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-pcie \
  > "$O/diag.out" 2> "$O/diag.err"
grep -c diag "$O/diag.out"
