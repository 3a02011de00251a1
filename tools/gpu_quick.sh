#!/bin/bash
# GPU tests + C3 / C2 bench; usage: bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-q}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$ROOT"
K=()
[ -n "${2:-}" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" \
  > "$O/gpu_tests.log" 2>&1
cd /tmp
timeout -k 10 300 python3 "$ROOT/bench.py" --workload c3 --steps 3 --warmup 1 > "$O/c3.json" 2> "$O/c3.err"
timeout -k 10 420 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
echo quick-done
