#!/bin/bash
# r4n: kernel trace of the C4 line (load and wakeups) and the level-0 place-pass diagnostics.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$ROOT/tools/gpu_r4.sh" "$1" kt4
bash "$ROOT/tools/gpu_ab2.sh" "$1/diag" - uigc-akka_amd/lib/ab/diag_nostore.so uigc-akka_amd/lib/ab/diag_noatomic.so
