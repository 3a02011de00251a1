#!/bin/bash
# Trace A/B (tools/ab_trace.py) + level log + quick bench; usage: bash tools/gpu_ab.sh <tag> [tests]
export CRGC_TEST_HOOKS=1  # the env variants below are test hooks (crgc_api.hip Knobs)
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-ab}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$ROOT"
if [ "${2:-}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
fi
cd /tmp
timeout -k 10 600 python3 "$ROOT/tools/ab_trace.py" --rounds 6 --variant BASE=0 --variant CRGC_ALPHA=0 \
  --variant CRGC_ALPHA=4 --variant CRGC_ALPHA=40 > "$O/ab.json" 2> "$O/ab.err"
CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 420 python3 "$ROOT/bench.py" --steps 2 --warmup 2 \
  --no-cpu-baseline > "$O/levels.json" 2> "$O/levels.err"
timeout -k 10 420 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
echo ab-done
