#!/bin/bash
# One measurement pass on the GPU box (run through gpurun):
#   bench.py (full default run, with the CPU baseline) -> $O/bench.json
#   rocprofv3 kernel trace + stats of a shorter bench   -> $O/kt/
#   rocprofv3 PMC passes FETCH_SIZE, WRITE_SIZE          -> $O/pmc_fetch/, $O/pmc_write/
# Every GPU step has its own time limit; steps are chained with &&.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 420 python3 "$ROOT/bench.py" > "$O/bench.json" 2> "$O/bench.err" &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_kt.json" 2> "$O/bench_kt.err" &&
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o pmc -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_fetch.json" 2> "$O/bench_fetch.err" &&
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o pmc -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_write.json" 2> "$O/bench_write.err"
echo measure-done
