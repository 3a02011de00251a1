#!/bin/bash
# Closure-mode check: variant parity tests, then the C2 bench with closure mode
# (default) and with the level BFS (CRGC_CLOSURE=0), and a kernel trace of the
# closure bench.  usage: bash tools/gpu_closure.sh <tag> [full]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-cl}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$ROOT"
if [ "${2:-}" = "full" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
else
  timeout -k 10 600 python -u -m pytest tests/test_hip_variants.py tests/test_hip_parity.py -m gpu -x -v \
    --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
fi
cd /tmp
timeout -k 10 420 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_cl.json" 2> "$O/bench_cl.err"
CRGC_CLOSURE=0 timeout -k 10 420 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline \
  > "$O/bench_lv.json" 2> "$O/bench_lv.err"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- \
  python3 "$ROOT/bench.py" --steps 4 --warmup 2 --no-cpu-baseline > "$O/bench_kt.json" 2> "$O/bench_kt.err"
echo closure-done
