#!/bin/bash
# C5 (DeltaGraph production + delta merge) profile; usage: bash tools/gpu_c5.sh <tag> [tests-k-expr]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-c5}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$ROOT"
if [ -n "${2:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$2" \
    > "$O/gpu_tests.log" 2>&1
fi
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- \
  python3 "$ROOT/bench.py" --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof_c5.json" 2> "$O/prof_c5.err"
timeout -k 10 420 python3 "$ROOT/bench.py" --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > "$O/c5.json" 2> "$O/c5.err"
CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 420 python3 "$ROOT/bench.py" --steps 3 --warmup 2 \
  --no-cpu-baseline > "$O/levels.json" 2> "$O/levels.err"
echo c5-done
