#!/bin/bash
# Full GPU suite, then tools/ab_bench.sh over the given variants.
# usage: bash tools/gpu_full_ab.sh <tag> <variant>...
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
shift
bash "$ROOT/tools/ab_bench.sh" "$TAG" "$@"
