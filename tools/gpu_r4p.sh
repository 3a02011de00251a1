#!/bin/bash
# r4p: the full GPU suite, the C4 line without the OpenMP leg (polling host waits),
# and the polling waits A/B'd on C2 (CRGC_SPIN_US=0: block at once).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$ROOT/tools/gpu_r4.sh" "$1" tests c4q
bash "$ROOT/tools/ab_env_wl.sh" "$1/spin" "c2" BASE CRGC_SPIN_US=0
