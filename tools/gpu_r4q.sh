#!/bin/bash
# r4q: C4 sub-merge size A/B (fewer capacity syncs per 1e7-entry wakeup), one pass each.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
mkdir -p "$O"
cd /tmp
for v in 2097152 4194304 1048576; do
  CRGC_TEST_HOOKS=1 CRGC_DEV_CHUNK=$v timeout -k 10 400 python3 -u "$ROOT/bench.py" --workload c4 --steps 5 --warmup 2 \
    --no-pcie --no-cpu-baseline > "$O/c4_chunk$v.json" 2> "$O/c4_chunk$v.err"
  python3 -c "import json; d=json.loads(open('$O/c4_chunk$v.json').read().strip().splitlines()[-1]); b=d['wakeup_breakdown_ms']; print('chunk $v', round(d['ms_per_step'],3), round(b['merge'],3), round(b['host_and_gaps'],3))" >> "$O/summary.txt"
done
cat "$O/summary.txt"
