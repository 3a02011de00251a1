#!/bin/bash
# Merge work: GPU tests (optional), kernel-trace profile of a short C2 bench, bench;
# usage: bash tools/gpu_merge.sh <tag> [tests]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-m}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$ROOT"
if [ "${2:-}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
fi
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- \
  python3 "$ROOT/bench.py" --steps 4 --warmup 2 --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof_bench.err"
timeout -k 10 420 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
echo merge-done
