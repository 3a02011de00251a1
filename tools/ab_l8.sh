#!/bin/bash
# Interleaved A/B of the logical-shard path over environment variants (each
# "K=V,K2=V2" or BASE), two passes: C2 or C4 (at half size) over 8 logical
# shards of the one GPU; ms per wakeup, the slowest shard's mark kernels,
# exchange and trace wall, rounds, into summary.txt.
# usage: bash tools/ab_l8.sh <tag> <c2|c4> <variant>...
export CRGC_TEST_HOOKS=1  # the env variants are test hooks (crgc_api.hip Knobs)
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-abl8}
WL=${2:-c2}
shift 2
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
extra=(--steps 5 --warmup 2)
[ "$WL" = c4 ] && extra=(--actors 50000000 --edges 500000000 --batch 5000000 --steps 3 --warmup 1)
for pass in 1 2; do
  for v in "$@"; do
    envs=()
    [ "$v" != "BASE" ] && IFS=',' read -ra envs <<< "$v"
    f="$O/p${pass}_$(echo "$v" | tr '=,/' '___').json"
    env "${envs[@]}" timeout -k 10 400 python3 "$ROOT/bench.py" --workload "$WL" --logical-shards 8 \
      --no-cpu-baseline "${extra[@]}" > "$f" 2>> "$O/err.log"
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); b=d['shard_breakdown_ms']; t=d['trace_shape']; print('$v', round(d['ms_per_step'],3), {k: round(x,3) for k, x in b.items()}, 'rounds', t['rounds'], 'xbytes', t['exchange_bytes'])" >> "$O/summary.txt"
  done
done
cat "$O/summary.txt"
