#!/bin/bash
# r4m: the final C2 bench line (OpenMP set parity, PCIe legs), C4 on one GPU (the scaling anchor),
# and the N > 1 code path rehearsed on one rank (nccl group, RCCL transport) at C2.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$ROOT/tools/gpu_r4.sh" "$1" rand c2 c4 c2rs
