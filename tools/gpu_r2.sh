#!/bin/bash
# Round-2 GPU check (run through gpurun): tests, smoke, C2 / C1 bench, level log,
# kernel trace.  usage: bash tools/gpu_r2.sh <tag> [skip-tests] [quick]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r2}
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$ROOT"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
fi
cd /tmp
CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 420 python3 "$ROOT/bench.py" --steps 3 --warmup 2 \
  --no-cpu-baseline > "$O/levels.json" 2> "$O/levels.err"
timeout -k 10 420 python3 "$ROOT/bench.py" --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
if [ "${3:-}" != "quick" ]; then
  timeout -k 10 300 python3 "$ROOT/bench.py" --workload c1 --steps 20 --warmup 5 > "$O/c1.json" 2> "$O/c1.err"
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_kt.json" 2> "$O/bench_kt.err"
fi
echo round-done
