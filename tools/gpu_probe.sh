#!/bin/bash
# HIP last-error / event / pointer-range semantics on the box: bash tools/gpu_probe.sh <tag>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 60 ./tools/_build/hip_probe > "$O/hip_probe.txt" 2>&1
cat "$O/hip_probe.txt"
