#!/bin/bash
# Full GPU suite, then the C5 bench and a kernel-trace profile of it (sqlite:
# profiles/dg_kernels.py reads it).  usage: bash tools/gpu_dg.sh <tag>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-dg}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
cd /tmp
timeout -k 10 420 python3 "$ROOT/bench.py" --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > "$O/c5.json" 2> "$O/c5.err"
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- \
  python3 "$ROOT/bench.py" --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof_c5.json" 2> "$O/prof_c5.err"
echo dg-done
