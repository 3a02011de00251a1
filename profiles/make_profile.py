"""Collect one GPU measurement directory (tools/gpu_run.sh output) into profiles/<tag>/.

usage: python profiles/make_profile.py gpurun_out/<run> profiles/<tag> [--pmc-latest]

Copies the bench lines, test / smoke logs and the level log, and reduces the
rocprofv3 outputs of the timed C2 wakeups (the profiled command runs
bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-pcie, so the last four
wakeups of the trace ARE the timed ones):
  c2_kernel_stats.csv      rocprofv3 --kernel-trace --stats summary (whole run)
  c2_steady_kernels.txt    last 24 dispatches per kernel (profiles/kt_summary.py)
  c2_per_wakeup.txt        device time per kernel per timed wakeup
  c2_pmc_steady.txt        FETCH_SIZE / WRITE_SIZE per launch over the last 4 wakeups
                           (two separate --pmc runs; profiles/pmc_summary.py)
--pmc-latest rewrites profiles/pmc_latest.json (what bench.py quotes as
`roofline.traffic`) from this run, naming it as the source.
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def run(args, out_path):
    r = subprocess.run([sys.executable] + args, capture_output=True, text=True, check=True)
    with open(out_path, "w") as f:
        f.write(r.stdout)
    return r.stdout


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    for name in ("gpu_tests.log", "smoke.log", "bench_c1.json", "bench_c2.json", "bench_c2q.json",
                 "bench_c3.json", "bench_c5.json", "bench_kt.json", "bench_fetch.json", "bench_write.json"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, name))
    lv = os.path.join(src, "levels.err")
    if os.path.exists(lv):
        with open(lv) as f, open(os.path.join(dst, "c2_levels.txt"), "w") as g:
            g.writelines(line for line in f if "[crgc] level" in line or "[bench]" in line)
    kt = os.path.join(src, "kt")
    if os.path.isdir(kt):
        shutil.copy(os.path.join(kt, "kt_kernel_stats.csv"), os.path.join(dst, "c2_kernel_stats.csv"))
        trace = os.path.join(kt, "kt_kernel_trace.csv")
        run([os.path.join(HERE, "kt_summary.py"), trace, "24"], os.path.join(dst, "c2_steady_kernels.txt"))
        run([os.path.join(HERE, "kt_summary.py"), trace, "4", "--wakeup"], os.path.join(dst, "c2_per_wakeup.txt"))
    fetch = os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv")
    write = os.path.join(src, "pmc_write", "pmc_counter_collection.csv")
    if os.path.exists(fetch) and os.path.exists(write):
        out = run([os.path.join(HERE, "pmc_summary.py"), "--last-wakeups", "4", fetch, write],
                  os.path.join(dst, "c2_pmc_steady.txt"))
        if "--pmc-latest" in sys.argv:
            kernels = json.loads(out.strip().splitlines()[-1])
            doc = {"source": f"{dst}/c2_pmc_steady.txt (rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, separate "
                             "runs of bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-pcie; dispatches of "
                             "the 4 timed wakeups; tools/gpu_run.sh pmc)",
                   "calibration": "profiles/r2d/calib_summary.txt (tools/calib_pmc.hip): FETCH_SIZE = 0.50 x "
                                  "bytes for 16-B and 8-B/lane streaming reads, 48-64 B per random 1-B read "
                                  "(line granularity), ~0 for L2-resident random 4-B probes",
                   "kernels": kernels}
            with open(os.path.join(HERE, "pmc_latest.json"), "w") as f:
                json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
