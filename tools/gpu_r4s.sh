#!/bin/bash
# r4s: sibling-supervisor dedupe (pull levels: supdedup; pull + push: supdedup2), checked
# against the trace parity tests, then A/B'd; then C4 with the OpenMP set comparison.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
mkdir -p "$O"
(cd "$ROOT" && CRGC_LIB_AB=$ROOT/uigc-akka_amd/lib/ab/supdedup2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
  --timeout 150 --timeout-method thread -k "bench_size or full_size or golden or parity or sharded" > "$O/dedup_tests.log" 2>&1)
tail -1 "$O/dedup_tests.log"
bash "$ROOT/tools/gpu_ab2.sh" "$1/ab" - uigc-akka_amd/lib/ab/supdedup.so uigc-akka_amd/lib/ab/supdedup2.so
bash "$ROOT/tools/gpu_r4.sh" "$1" c4
