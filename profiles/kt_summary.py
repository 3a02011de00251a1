"""Per-kernel durations from a rocprofv3 rocpd database, restricted to the last
K dispatches of each kernel (the bench's steady-state wakeups).
usage: python profiles/kt_summary.py <run_results.db> [K]"""
import sqlite3
import sys
from collections import defaultdict

db, K = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4
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
