#!/bin/bash
# PCIe-inclusive C2 wakeups (bench.py's pcie_inclusive) under host-batch variants:
#   bash tools/gpu_pcie.sh <tag> <variant>...   (variant: BASE or K=V[,K2=V2])
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  envs=()
  [ "$v" != "BASE" ] && IFS=',' read -ra envs <<< "$v"
  f="$O/$(echo "$v" | tr '=,/' '___').json"
  env "${envs[@]}" timeout -k 10 300 python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$f" 2>> "$O/err.log"
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); p=d['pcie_inclusive']; print('$v', round(d['ms_per_step'],3), {k: (round(x,3) if isinstance(x,float) else x) for k,x in p.items() if k!='note'})" >> "$O/summary.txt"
done
cat "$O/summary.txt"
