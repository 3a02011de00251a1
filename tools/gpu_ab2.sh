#!/bin/bash
# A/B of builds against the in-tree one (run through gpurun from the repo root):
#   bash tools/gpu_ab2.sh <tag> <tests-expr|-> <lib.so>...
# 1. pytest -m gpu on the in-tree build (-k <tests-expr>, "all" for the whole
#    suite, "-" to skip);
# 2. C2 benches alternating the in-tree build ("new") and every given .so, two
#    passes (summary.txt: variant, ms per wakeup, merge ms, mark-kernel ms);
# 3. one C2 level log per build (CRGC_LEVEL_LOG, all level kernels timed).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$1
K=$2
shift 2
mkdir -p "$O"
export TMPDIR=/tmp
if [ "$K" != "-" ]; then
  sel=()
  [ "$K" != all ] && sel=(-k "$K")
  (cd "$ROOT" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 \
    --timeout-method thread "${sel[@]}" > "$O/gpu_tests.log" 2>&1)
  tail -1 "$O/gpu_tests.log"
fi
cd /tmp
libs=(new "$@")
for pass in 1 2; do
  for v in "${libs[@]}"; do
    n=$(basename "$v" .so)
    envs=()
    [ "$v" != new ] && envs=(CRGC_LIB_AB=$ROOT/$v)
    f="$O/p${pass}_$n.json"
    env "${envs[@]}" timeout -k 10 300 python3 "$ROOT/bench.py" --steps 15 --warmup 3 --no-cpu-baseline --no-pcie \
      > "$f" 2>> "$O/err.log"
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); b=d['wakeup_breakdown_ms']; print('$n', round(d['ms_per_step'],4), round(b['merge'],4), round(b['mark_kernels'],4))" >> "$O/summary.txt"
  done
done
cat "$O/summary.txt"
for v in "${libs[@]}"; do
  n=$(basename "$v" .so)
  envs=()
  [ "$v" != new ] && envs=(CRGC_LIB_AB=$ROOT/$v)
  env "${envs[@]}" CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 300 python3 "$ROOT/bench.py" \
    --steps 4 --warmup 2 --no-cpu-baseline --no-pcie > "$O/levels_$n.json" 2> "$O/levels_$n.err"
done
echo "[gpu_ab2] done"
