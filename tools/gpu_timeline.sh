#!/bin/bash
# Kernel trace of a short default C2 bench and the timeline of its last wakeup
# (profiles/timeline.py: idle gap before each kernel).  usage: bash tools/gpu_timeline.sh <tag>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-tl}
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- \
  python3 "$ROOT/bench.py" --steps 4 --warmup 2 --no-cpu-baseline > "$O/bench_kt.json" 2> "$O/bench_kt.err"
python3 "$ROOT/profiles/timeline.py" "$O/kt/kt_kernel_trace.csv" > "$O/timeline.txt"
echo timeline-done
