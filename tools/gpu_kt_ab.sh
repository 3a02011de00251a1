#!/bin/bash
# GPU suite on the in-tree build, then a kernel trace of a short C2 bench for
# each of two builds (twice, interleaved): usage: bash tools/gpu_kt_ab.sh <tag> <base.so> <new.so>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-ktab}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest "$ROOT/tests" -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$O/tests.log" 2>&1
echo tests-done
cd /tmp
for pass in 1 2; do
  for v in base new; do
    lib=$2
    [ "$v" = new ] && lib=$3
    CRGC_LIB_AB=$ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$v$pass" -o kt -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$O/$v$pass.json" 2> "$O/$v$pass.err"
    echo "$v$pass done"
  done
done
