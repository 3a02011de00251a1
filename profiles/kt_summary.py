"""Per-kernel durations from a rocprofv3 rocpd database, restricted to the last
K dispatches of each kernel (the bench's steady-state wakeups).
usage: python profiles/kt_summary.py <run_results.db | kernel_trace.csv> [K] [--wakeup]"""
import sqlite3
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
db, K = args[0], int(args[1]) if len(args) > 1 else 4
if db.endswith(".csv"):  # rocprofv3 --output-format csv kernel_trace.csv
    import csv
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"])) for r in csv.DictReader(open(db))),
                  key=lambda x: x[1])
else:
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
by = defaultdict(list)
for name, s, e, gx, wx in rows:
    by[name].append((e - s, gx // max(wx, 1)))
out = []
for name, v in by.items():
    last = v[-K:]
    out.append((sum(d for d, _ in last) / len(last) / 1000.0, len(v), last[-1][1], name))
for us, n, wg, name in sorted(out, reverse=True)[:40]:
    print(f"{us:9.1f} us  x{n:<5d} wg={wg:<7d} {name[:90]}")


def per_wakeup(rows, K):
    """Kernel time per wakeup: dispatches between consecutive k_sweep_gather
    ends (one merge + one trace each), averaged over the last K wakeups."""
    ends = [e for name, s, e, *_ in rows if "k_sweep_gather" in name]
    acc = defaultdict(float)
    for lo, hi in zip(ends[-K - 1:-1], ends[-K:]):
        for name, s, e, *_ in rows:
            if lo < e <= hi:
                acc[name] += (e - s) / 1000.0 / K
    return acc


if "--wakeup" in sys.argv:
    acc = per_wakeup(rows, K)
    print(f"\nper wakeup (last {K}): total {sum(acc.values()):.1f} us")
    for name, us in sorted(acc.items(), key=lambda x: -x[1])[:30]:
        print(f"{us:9.1f} us  {name[:90]}")
