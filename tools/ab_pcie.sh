#!/bin/bash
# Interleaved A/B of env variants (each "K=V,K2=V2" or BASE) on the C2 line's
# PCIe-inclusive legs (pageable, registered, drain loop), two passes; per
# variant the registered wakeup, its merge call, and the drain loop by chunk
# size into summary.txt.
# usage: bash tools/ab_pcie.sh <tag> <variant>...
export CRGC_TEST_HOOKS=1
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-abp}
shift
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for pass in 1 2; do
  for v in "$@"; do
    envs=()
    [ "$v" != "BASE" ] && IFS=',' read -ra envs <<< "$v"
    f="$O/p${pass}_$(echo "$v" | tr '=,/' '___').json"
    env "${envs[@]}" timeout -k 10 300 python3 "$ROOT/bench.py" --steps 6 --warmup 2 --no-cpu-baseline \
      > "$f" 2>> "$O/err.log"
    python3 -c "
import json
d = json.loads(open('$f').read().strip().splitlines()[-1])
p = d['pcie_inclusive']; r = p['registered']; dl = p['drain_loop']
print('$v', 'pageable', round(p['ms_per_wakeup'], 3), 'registered', round(r['ms_per_wakeup'], 3),
      'merge_call', round(r['merge_call_ms'], 3), 'pack', round(r['pack_ms_per_wakeup'], 3),
      'drain', round(dl['ms_per_wakeup'], 3), dl['ms_by_chunk_entries'])" >> "$O/summary.txt"
  done
done
cat "$O/summary.txt"
