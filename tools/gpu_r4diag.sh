#!/bin/bash
# Diagnostic builds (results wrong on purpose: no parity checks run): the level-0
# place pass without its bin stores, and without its LDS position atomics.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$ROOT/tools/gpu_ab2.sh" "$1" - uigc-akka_amd/lib/ab/diag_nostore.so uigc-akka_amd/lib/ab/diag_noatomic.so
