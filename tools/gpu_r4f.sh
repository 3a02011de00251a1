#!/bin/bash
# r4f: kernel trace of the timed C2 wakeups, the random-access probe, and the
# k_tail takeover threshold A/B (C2, C1) — one gpurun call.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$ROOT/tools/gpu_r4.sh" "$1" kt rand
bash "$ROOT/tools/ab_env_wl.sh" "$1/tail" "c2 c1" BASE CRGC_TAIL_START=32768
