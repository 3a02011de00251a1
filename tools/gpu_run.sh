#!/bin/bash
# GPU driver (run through gpurun from the repo root):
#   bash tools/gpu_run.sh <tag> <steps...>
# steps (each under its own time limit, chained: the first failure ends the call):
#   tests[:-k expr]  pytest -m gpu (optionally -k)        smoke   __graft_entry__.smoke()
#   c2 c1 c3 c5      bench.py lines                        levels  C2 level log (CRGC_LEVEL_LOG)
#   c2d              the driver's N = 1 command (--gpus 1 --steps 20 --warmup 5)
#   kt               rocprofv3 --kernel-trace --stats of the timed C2 wakeups only (--no-pcie)
#   ktp              the same with the PCIe-inclusive wakeups (pageable, then registered host batches) at the end
#   pmc              FETCH_SIZE and WRITE_SIZE passes of the same command, one run each
#   probe            tools/hip_probe.hip: HIP last-error / event / pointer-range semantics
#   rand             tools/rand_probe.hip: random-access ceilings (loads, atomics, CAS, stores)
#   evprobe          tools/event_probe.hip: the idle GPU time a timing event costs between launches
#   c4               C4 unsharded on one GPU (1e8 actors / 1e9 edges, the scaling anchor)
#   c4q              the C4 line without the OpenMP leg (no set comparison)
#   kt4              kernel trace of the C4 N = 1 line (load and wakeups)
#   c4l8 c2l8        C4 (at half size: 8 proxy-heavy shards of the full graph need > 288 GB) / C2 over
#                    8 logical shards on the one GPU (the sharded protocol at scale)
#   c2rs c4rs        the N>1 bench path itself on one rank (nccl group, RCCL transport, one shard)
#   ktrs             kernel trace of c2rs
#   ktl8             kernel trace of c4l8 (every shard's kernels, one process)
#   ktl8s            ktl8 with every shard on one stream (--shared-stream): the shards' kernels run one at
#                    a time, so each duration is the kernel's own and their sum is the GPU work per wakeup
#   kt2l8s           the same for C2 over 8 logical shards
#   c4l8s c2l8s      logical shards on one shared stream with the per-shard level log (all level kernels timed)
#   c2l8x<k> c4l8x<k>  c2l8 / c4l8 with mark rounds capped at k levels (CRGC_XLEVELS, test hook)
#   lv:<variants>    per-level kernel times (CRGC_KERNEL_TIMING=2) over env variants, two passes (tools/lv_summary.py)
#   ab:<variants>    tools/ab_bench.sh A/B of env variants on the C2 line
#   abl:<variants>   the same after 100 warmup wakeups (a grown graph)
#   abp:<variants>   tools/ab_pcie.sh A/B of env variants on the PCIe-inclusive legs (registered, drain loop)
#   ab2l8:<variants> ab4l8:<variants>  tools/ab_l8.sh A/B of env variants on C2 / C4 logical shards
#   longkt           kernel trace + level log of the long run
#   long             C2 over 200 wakeups: the steady state, rebuilds / repacks amortized in
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
B="python3 $ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-pcie"
for step in "$@"; do
  echo "[gpu_r4] $step $(date +%T)"
  case "$step" in
    tests|tests:*)
      K=()
      [ "$step" != tests ] && K=(-k "${step#tests:}")
      (cd "$ROOT" && timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 150 \
        --timeout-method thread "${K[@]}" > "$O/gpu_tests.log" 2>&1) ;;
    smoke) (cd "$ROOT" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1) ;;
    c2) (cd /tmp && timeout -k 10 480 python3 "$ROOT/bench.py" > "$O/bench_c2.json" 2> "$O/bench_c2.err") ;;
    c2d) (cd /tmp && timeout -k 10 600 python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 \
          > "$O/bench_c2d.json" 2> "$O/bench_c2d.err") ;;  # the driver's own N = 1 command
    c2q) (cd /tmp && timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline > "$O/bench_c2q.json" 2> "$O/bench_c2q.err") ;;
    c1) (cd /tmp && timeout -k 10 300 python3 "$ROOT/bench.py" --workload c1 > "$O/bench_c1.json" 2> "$O/bench_c1.err") ;;
    c3) (cd /tmp && timeout -k 10 300 python3 "$ROOT/bench.py" --workload c3 > "$O/bench_c3.json" 2> "$O/bench_c3.err") ;;
    c5) (cd /tmp && timeout -k 10 420 python3 "$ROOT/bench.py" --workload c5 --steps 5 --warmup 2 --no-cpu-baseline \
          > "$O/bench_c5.json" 2> "$O/bench_c5.err") ;;
    levels) (cd /tmp && CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 420 $B --timing-every 1 > "$O/levels.json" 2> "$O/levels.err") ;;
    kt) (cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- $B \
          > "$O/bench_kt.json" 2> "$O/bench_kt.err") ;;
    ktp) (cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktp" -o kt -- \
          python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/bench_ktp.json" 2> "$O/bench_ktp.err") ;;
    pmc) (cd /tmp && timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o pmc -- $B \
            > "$O/bench_fetch.json" 2> "$O/bench_fetch.err" &&
          timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o pmc -- $B \
            > "$O/bench_write.json" 2> "$O/bench_write.err") ;;
    probe) (cd "$ROOT" && timeout -k 10 60 ./tools/_build/hip_probe > "$O/hip_probe.txt" 2>&1) ;;
    rand) (cd "$ROOT" && timeout -k 10 120 ./tools/_build/rand_probe > "$O/rand_probe.txt" 2>&1) ;;
    evprobe) (cd "$ROOT" && timeout -k 10 60 ./tools/_build/event_probe > "$O/event_probe.txt" 2>&1) ;;
    c4) (cd /tmp && CRGC_LEVEL_LOG=1 timeout -k 10 1000 python3 -u "$ROOT/bench.py" --workload c4 --steps 5 \
          --warmup 2 --no-pcie > "$O/bench_c4.json" 2> "$O/bench_c4.err") ;;
    c4q) (cd /tmp && timeout -k 10 900 python3 -u "$ROOT/bench.py" --workload c4 --steps 5 --warmup 2 --no-pcie \
          --no-cpu-baseline > "$O/bench_c4q.json" 2> "$O/bench_c4q.err") ;;
    kt4) (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt4" -o kt -- \
          python3 "$ROOT/bench.py" --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie \
          > "$O/bench_kt4.json" 2> "$O/bench_kt4.err") ;;
    c4l8) (cd /tmp && CRGC_LEVEL_LOG=1 timeout -k 10 1000 python3 -u "$ROOT/bench.py" --workload c4 --logical-shards 8 \
          --actors 50000000 --edges 500000000 --batch 5000000 \
          --steps 3 --warmup 1 > "$O/bench_c4l8.json" 2> "$O/bench_c4l8.err") ;;
    c4l8s|c2l8s)  # the logical-shard run on one shared stream with the level log (every level kernel timed)
      wl=${step%%l8s}; extra=(--steps 3 --warmup 1)
      [ "$wl" = c4 ] && extra=(--actors 50000000 --edges 500000000 --batch 5000000 --steps 2 --warmup 1)
      (cd /tmp && CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 timeout -k 10 600 python3 -u "$ROOT/bench.py" --workload $wl \
          --logical-shards 8 --shared-stream --no-cpu-baseline "${extra[@]}" > "$O/bench_${step}.json" \
          2> "$O/bench_${step}.err") ;;
    c2rs) (cd /tmp && timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
          --master-addr=127.0.0.1 --master-port=29517 "$ROOT/bench.py" --gpus 1 --workload c2 --rehearse-sharded \
          --steps 5 --warmup 2 --no-pcie > "$O/bench_c2rs.json" 2> "$O/bench_c2rs.err") ;;
    ktrs) (cd /tmp && MASTER_ADDR=127.0.0.1 MASTER_PORT=29519 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 \
          timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrs" -o kt -- \
          python3 -u "$ROOT/bench.py" --gpus 1 --workload c2 --rehearse-sharded --steps 5 --warmup 2 \
          --no-pcie --no-cpu-baseline > "$O/bench_ktrs.json" 2> "$O/bench_ktrs.err") ;;  # (the rank itself, no launcher)
    c4rs) (cd /tmp && timeout -k 10 1000 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
          --master-addr=127.0.0.1 --master-port=29518 "$ROOT/bench.py" --gpus 1 --workload c4 --rehearse-sharded \
          --steps 3 --warmup 1 --no-pcie --no-cpu-baseline > "$O/bench_c4rs.json" 2> "$O/bench_c4rs.err") ;;
    c2l8) (cd /tmp && timeout -k 10 600 python3 -u "$ROOT/bench.py" --workload c2 --logical-shards 8 \
          --steps 5 --warmup 2 > "$O/bench_c2l8.json" 2> "$O/bench_c2l8.err") ;;
    c2l8log) (cd /tmp && CRGC_LEVEL_LOG=1 timeout -k 10 600 python3 -u "$ROOT/bench.py" --workload c2 --logical-shards 8 \
          --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_c2l8log.json" 2> "$O/bench_c2l8log.err") ;;
    c2l8x*|c4l8x*)  # the same with CRGC_XLEVELS=<k> (mark rounds capped at k levels; a test hook)
      k=${step#*x}; wl=${step%%l8x*}
      extra=()
      [ "$wl" = c4 ] && extra=(--actors 50000000 --edges 500000000 --batch 5000000 --steps 3 --warmup 1)
      [ "$wl" = c2 ] && extra=(--steps 5 --warmup 2 --no-cpu-baseline)
      (cd /tmp && CRGC_TEST_HOOKS=1 CRGC_XLEVELS=$k timeout -k 10 600 python3 -u "$ROOT/bench.py" --workload $wl \
          --logical-shards 8 "${extra[@]}" > "$O/bench_${step}.json" 2> "$O/bench_${step}.err") ;;
    ktl8) (cd /tmp && timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktl8" -o kt -- \
          python3 -u "$ROOT/bench.py" --workload c4 --logical-shards 8 \
          --actors 50000000 --edges 500000000 --batch 5000000 --no-cpu-baseline \
          --steps 2 --warmup 1 > "$O/bench_ktl8.json" 2> "$O/bench_ktl8.err") ;;
    ktl8s) (cd /tmp && timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$O/ktl8s" -o kt -- python3 -u "$ROOT/bench.py" --workload c4 --logical-shards 8 --shared-stream \
          --actors 50000000 --edges 500000000 --batch 5000000 --no-cpu-baseline \
          --steps 2 --warmup 1 > "$O/bench_ktl8s.json" 2> "$O/bench_ktl8s.err") ;;
    kt2l8s|kt2l8s:*)  # kt2l8s:K=V,K2=V2 runs it under those (test-hook) env settings
      envs=(CRGC_TEST_HOOKS=1); sfx=""
      if [ "$step" != kt2l8s ]; then IFS=',' read -ra ev <<< "${step#*:}"; envs+=("${ev[@]}"); sfx="_$(echo "${step#*:}" | tr '=,/' '___')"; fi
      (cd /tmp && env "${envs[@]}" timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$O/kt2l8s$sfx" -o kt -- python3 -u "$ROOT/bench.py" --workload c2 --logical-shards 8 --shared-stream \
          --no-cpu-baseline \
          --steps 4 --warmup 2 > "$O/bench_kt2l8s$sfx.json" 2> "$O/bench_kt2l8s$sfx.err") ;;
    lv:*)  # per-level kernel times (all three level kernels timed) over env variants, two passes
      read -ra vs <<< "${step#*:}"
      for pass in 1 2; do
        for v in "${vs[@]}"; do
          envs=(CRGC_TEST_HOOKS=1 CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2)
          [ "$v" != "BASE" ] && IFS=',' read -ra ev <<< "$v" && envs+=("${ev[@]}")
          f="$O/lv_p${pass}_$(echo "$v" | tr '=,/' '___')"
          (cd /tmp && env "${envs[@]}" timeout -k 10 300 $B --timing-every 1 > "$f.json" 2> "$f.err")
          { echo "== pass $pass $v"; python3 "$ROOT/tools/lv_summary.py" "$f.err" 3; } >> "$O/lv_summary.txt"
        done
      done ;;
    ab:*)  # tools/ab_bench.sh (C2 N = 1) over the variants after the colon (separated by spaces)
      read -ra vs <<< "${step#*:}"
      (cd "$ROOT" && bash tools/ab_bench.sh "$TAG/ab_c2" "${vs[@]}" > /dev/null) ;;
    abl:*)  # the same after 100 warmup wakeups (the live set grown to ~2.1e7: the long run's middle)
      read -ra vs <<< "${step#*:}"
      (cd "$ROOT" && AB_ARGS="--steps 10 --warmup 100" bash tools/ab_bench.sh "$TAG/ab_c2l" "${vs[@]}" > /dev/null) ;;
    abp:*)  # tools/ab_pcie.sh: the PCIe-inclusive legs (pageable, registered, drain loop) over env variants
      read -ra vs <<< "${step#*:}"
      (cd "$ROOT" && bash tools/ab_pcie.sh "$TAG/ab_pcie" "${vs[@]}" > /dev/null) ;;
    ab2l8:*|ab4l8:*)  # tools/ab_l8.sh over the variants after the colon (separated by spaces)
      wl=${step%%l8:*}; wl=c${wl#ab}
      read -ra vs <<< "${step#*:}"
      (cd "$ROOT" && bash tools/ab_l8.sh "$TAG/ab_${wl}l8" "$wl" "${vs[@]}" > /dev/null) ;;
    longkt) (cd /tmp && CRGC_LEVEL_LOG=1 timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$O/longkt" -o kt -- python3 -u "$ROOT/bench.py" --steps 200 --warmup 2 --no-pcie --no-cpu-baseline \
          > "$O/bench_longkt.json" 2> "$O/bench_longkt.err") ;;
    long) (cd /tmp && timeout -k 10 900 python3 -u "$ROOT/bench.py" --steps 200 --warmup 2 --no-pcie \
          --no-cpu-baseline > "$O/bench_long.json" 2> "$O/bench_long.err") ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_r4] done $(date +%T)"
