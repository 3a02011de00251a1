#!/bin/bash
# Counter calibration + steady-state PMC passes of the C2 bench (gpurun).
# usage: bash tools/gpu_calib.sh <tag>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-calib}
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
CAL=$ROOT/tools/_build/calib_pmc
timeout -k 10 120 "$CAL" > "$O/calib.jsonl" 2> "$O/calib.err"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/calib_kt" -o kt -- "$CAL" > /dev/null 2>> "$O/calib.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/calib_fetch" -o pmc -- "$CAL" > /dev/null 2>> "$O/calib.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/calib_write" -o pmc -- "$CAL" > /dev/null 2>> "$O/calib.err"
B="python3 $ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline"
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- $B > "$O/bench_kt.json" 2> "$O/bench_kt.err"
timeout -k 10 480 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o pmc -- $B > "$O/bench_fetch.json" 2> "$O/bench_fetch.err"
timeout -k 10 480 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o pmc -- $B > "$O/bench_write.json" 2> "$O/bench_write.err"
echo calib-done
