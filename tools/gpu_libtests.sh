#!/bin/bash
# pytest -m gpu against another build (CRGC_LIB_AB): bash tools/gpu_libtests.sh <tag> <lib.so> [-k expr]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
LIB=$2
shift 2
mkdir -p "$O"
cd "$ROOT"
CRGC_LIB_AB=$ROOT/$LIB timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 \
  --timeout-method thread "$@" > "$O/gpu_tests_$(basename "$LIB" .so).log" 2>&1
tail -1 "$O/gpu_tests_$(basename "$LIB" .so).log"
