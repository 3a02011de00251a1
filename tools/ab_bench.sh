#!/bin/bash
# Interleaved bench A/B over environment variants (each "K=V,K2=V2" or BASE),
# two passes; ms_per_step, merge and mark per variant into summary.txt.
# usage: [AB_ARGS="--steps K --warmup W"] bash tools/ab_bench.sh <tag> <variant>...
export CRGC_TEST_HOOKS=1  # the env variants below are test hooks (crgc_api.hip Knobs)
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-abb}
shift
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for pass in 1 2; do
  for v in "$@"; do
    envs=()
    [ "$v" != "BASE" ] && IFS=',' read -ra envs <<< "$v"
    f="$O/p${pass}_$(echo "$v" | tr '=,/' '___').json"
    env "${envs[@]}" timeout -k 10 300 python3 "$ROOT/bench.py" ${AB_ARGS:---steps 15 --warmup 3} --no-cpu-baseline --no-pcie \
      > "$f" 2>> "$O/err.log"
    python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); b=d['wakeup_breakdown_ms']; print('$v', round(d['ms_per_step'],4), round(b['merge'],4), round(b['mark_kernels'],4))" >> "$O/summary.txt"
  done
done
cat "$O/summary.txt"
