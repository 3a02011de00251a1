#!/bin/bash
# A/B: C2 bench with and without a compaction after the load, level logs
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-cmp}
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 420 python3 "$ROOT/bench.py" --steps 3 --warmup 2 \
  --no-cpu-baseline --compact > "$O/levels_compact.json" 2> "$O/levels_compact.err"
timeout -k 10 420 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --compact > "$O/bench_compact.json" 2> "$O/bench_compact.err"
timeout -k 10 420 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
echo cmp-done
