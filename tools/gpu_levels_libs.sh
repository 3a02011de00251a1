#!/bin/bash
# C2 level logs (all level kernels timed) of the in-tree build and of other builds:
#   bash tools/gpu_levels_libs.sh <tag> <lib.so>...
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for v in new "$@"; do
  n=$(basename "$v" .so)
  envs=()
  [ "$v" != new ] && envs=(CRGC_LIB_AB=$ROOT/$v)
  env "${envs[@]}" CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 240 python3 "$ROOT/bench.py" \
    --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > "$O/levels_$n.json" 2> "$O/levels_$n.err"
  echo "$n rc=$?"
done
