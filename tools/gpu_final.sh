#!/bin/bash
# End-of-round measurement (gpurun), in two parts so each fits one call:
#   bash tools/gpu_final.sh <tag> A   GPU tests, smoke, C2 level log, C2 / C1 / C3 / C5 benches
#   bash tools/gpu_final.sh <tag> B   kernel trace + steady-state FETCH_SIZE / WRITE_SIZE passes of C2
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-final}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$ROOT"
if [ "${2:-A}" = "A" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  cd /tmp
  CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 420 python3 "$ROOT/bench.py" --steps 3 --warmup 2 \
    --no-cpu-baseline > "$O/levels.json" 2> "$O/levels.err"
  timeout -k 10 420 python3 "$ROOT/bench.py" > "$O/bench_c2.json" 2> "$O/bench_c2.err"
  timeout -k 10 300 python3 "$ROOT/bench.py" --workload c1 > "$O/bench_c1.json" 2> "$O/bench_c1.err"
  timeout -k 10 300 python3 "$ROOT/bench.py" --workload c3 > "$O/bench_c3.json" 2> "$O/bench_c3.err"
  timeout -k 10 420 python3 "$ROOT/bench.py" --workload c5 --steps 5 --warmup 2 --no-cpu-baseline \
    > "$O/bench_c5.json" 2> "$O/bench_c5.err"
else
  cd /tmp
  B="python3 $ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline"
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- $B \
    > "$O/bench_kt.json" 2> "$O/bench_kt.err"
  timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o pmc -- $B \
    > "$O/bench_fetch.json" 2> "$O/bench_fetch.err"
  timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o pmc -- $B \
    > "$O/bench_write.json" 2> "$O/bench_write.err"
fi
echo final-done
