#!/bin/bash
# Per-dispatch HBM counters of one C2 trace (tools/ab_trace.py, one round):
# separate rocprofv3 passes for FETCH_SIZE, WRITE_SIZE and the L2 hit counters.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-r1}/tprof
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for pass in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo "$pass" | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$O/$name" -o p -- \
    python3 "$ROOT/tools/ab_trace.py" --rounds 1 --wakeups 1 > "$O/$name.json" 2> "$O/$name.err"
done
echo prof-done
