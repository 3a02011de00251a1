#!/bin/bash
# r4o: the wave-sorted bin stores (wsort.so) checked against the binned-level
# parity tests, then A/B'd with the place-grid variants against the in-tree build.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
mkdir -p "$O"
(cd "$ROOT" && CRGC_LIB_AB=$ROOT/uigc-akka_amd/lib/ab/wsort.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
  --timeout 150 --timeout-method thread -k "bench_size or full_size or golden" > "$O/wsort_tests.log" 2>&1)
tail -1 "$O/wsort_tests.log"
bash "$ROOT/tools/gpu_ab2.sh" "$1/ab" - uigc-akka_amd/lib/ab/wsort.so uigc-akka_amd/lib/ab/wg256.so \
  uigc-akka_amd/lib/ab/wg1024.so
bash "$ROOT/tools/gpu_r4.sh" "$1" c4q
