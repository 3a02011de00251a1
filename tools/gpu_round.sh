#!/bin/bash
# Round check on the GPU box (run through gpurun):
#   pytest -m gpu, smoke(), bench.py C2 (default run incl. cpu_baseline), C3 bench,
#   rocprofv3 --kernel-trace --stats of a short C2 bench, optional FETCH_SIZE / WRITE_SIZE passes.
# Every GPU step has its own limit; steps are chained with && so the first failure ends it.
# usage: bash tools/gpu_round.sh <tag> [skip-tests] [pmc]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
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
timeout -k 10 420 python3 "$ROOT/bench.py" > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 python3 "$ROOT/bench.py" --workload c3 --steps 3 --warmup 1 > "$O/c3.json" 2> "$O/c3.err"
timeout -k 10 420 python3 "$ROOT/bench.py" --workload c5 --steps 5 --warmup 1 > "$O/c5.json" 2> "$O/c5.err"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_kt.json" 2> "$O/bench_kt.err"
if [ "${3:-}" = "pmc" ]; then
  timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o pmc -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_fetch.json" 2> "$O/bench_fetch.err"
  timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o pmc -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_write.json" 2> "$O/bench_write.err"
fi
echo round-done
