#!/bin/bash
# r4j: binned-level tests, k_bin_apply A/B (two workgroups per bin vs place1's one),
# the full C2 bench line (OpenMP set parity, PCIe legs), C4 over 8 logical shards at half size.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$ROOT/tools/gpu_r4.sh" "$1" "tests:bench_size or full_size or parity"
bash "$ROOT/tools/gpu_ab2.sh" "$1/ab" - uigc-akka_amd/lib/ab/place1.so
bash "$ROOT/tools/gpu_r4.sh" "$1" c2 c4l8
