#!/bin/bash
# GPU parity tests, then an interleaved push/pull A/B and a per-level log.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-r1}
mkdir -p "$O"
timeout -k 10 600 python -m pytest tests -m gpu -q -x > "$O/gpu_tests.log" 2>&1 &&
timeout -k 10 400 python tools/ab_trace.py --rounds 6 --variant CRGC_PULL=0 \
  --variant CRGC_PULL=1,CRGC_PULL_DIV=16 --variant CRGC_PULL=1,CRGC_PULL_DIV=32 \
  --variant CRGC_PULL=1,CRGC_PULL_DIV=64 > "$O/ab_pull.json" 2> "$O/ab_pull.err" &&
CRGC_LEVEL_LOG=1 timeout -k 10 300 python tools/ab_trace.py --rounds 1 --variant CRGC_PULL=0 \
  --variant CRGC_PULL=1 > "$O/levels.json" 2> "$O/levels.err"
