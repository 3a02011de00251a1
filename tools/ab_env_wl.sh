#!/bin/bash
# Env-variant A/B over workloads, two interleaved passes:
#   bash tools/ab_env_wl.sh <tag> "<workloads>" <variant>...   (variant: BASE or K=V[,K2=V2])
# summary.txt: workload, variant, ms per wakeup (C3: per trace), mark-kernel ms
export CRGC_TEST_HOOKS=1  # the env variants below are test hooks (crgc_api.hip Knobs)
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
WLS=$2
shift 2
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for pass in 1 2; do
  for wl in $WLS; do
    for v in "$@"; do
      envs=()
      [ "$v" != "BASE" ] && IFS=',' read -ra envs <<< "$v"
      f="$O/p${pass}_${wl}_$(echo "$v" | tr '=,/' '___').json"
      env "${envs[@]}" timeout -k 10 300 python3 "$ROOT/bench.py" --workload "$wl" --steps 10 --warmup 3 \
        --no-cpu-baseline --no-pcie > "$f" 2>> "$O/err.log"
      python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); b=d.get('wakeup_breakdown_ms', {}); print('$wl', '$v', round(d['ms_per_step'],4), round(b.get('mark_kernels', 0),4))" >> "$O/summary.txt"
    done
  done
done
cat "$O/summary.txt"
