#!/bin/bash
# GPU parity tests, C3 with and without k_tail, C2 A/B with the per-level log.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-r1}
mkdir -p "$O"
timeout -k 10 700 python -m pytest tests -m gpu -q -x > "$O/gpu_tests.log" 2>&1 &&
CRGC_TAIL=1 timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 > "$O/c3_tail.json" 2> "$O/c3_tail.err" &&
CRGC_TAIL=0 timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 0 --no-cpu-baseline > "$O/c3_notail.json" 2> "$O/c3_notail.err" &&
timeout -k 10 400 python tools/ab_trace.py --rounds 6 --variant CRGC_TAIL=0 --variant CRGC_TAIL=1 \
  > "$O/ab_tail.json" 2> "$O/ab_tail.err" &&
CRGC_LEVEL_LOG=1 timeout -k 10 300 python tools/ab_trace.py --rounds 1 --variant CRGC_TAIL=1 \
  > "$O/levels.json" 2> "$O/levels.err"
