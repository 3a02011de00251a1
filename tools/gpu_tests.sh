#!/bin/bash
# GPU parity tests only (optionally a -k filter): bash tools/gpu_tests.sh <tag> [pytest -k expr]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-r1}
mkdir -p "$O"
cd "$ROOT"
K=()
[ -n "${2:-}" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" \
  > "$O/gpu_tests.log" 2>&1
echo tests-done
