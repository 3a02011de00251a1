#!/bin/bash
# Kernel trace of a short C2 bench plus FETCH_SIZE / WRITE_SIZE passes, and a
# per-level log of the bench's own traces.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-r1}/bprof
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
CRGC_LEVEL_LOG=1 timeout -k 10 300 python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/levels.json" 2> "$O/levels.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$O/kt.json" 2> "$O/kt.err"
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$O/$pass" -o p -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/$pass.json" 2> "$O/$pass.err"
done
echo prof-done
