#!/bin/bash
# r4n: kernel trace of the C4 line (load and wakeups) and the place-grid A/B (256 / 512 / 1024 workgroups).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$ROOT/tools/gpu_r4.sh" "$1" kt4
bash "$ROOT/tools/gpu_ab2.sh" "$1/ab" - uigc-akka_amd/lib/ab/wg256.so uigc-akka_amd/lib/ab/wg1024.so
