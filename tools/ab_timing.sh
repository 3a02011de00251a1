set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/abt
mkdir -p $O
cd /tmp
for t in 1 0 1 0; do
  CRGC_KERNEL_TIMING=$t timeout -k 10 300 python3 $ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/t$t.json 2>> $O/err.log
  python3 -c "import json; d=json.loads(open('$O/t$t.json').read().strip().splitlines()[-1]); print('timing=$t', d['ms_per_step'], d['wakeup_breakdown_ms']['mark_kernels'])" >> $O/summary.txt
done
cat $O/summary.txt
