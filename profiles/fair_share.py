"""Busy time of a multi-stream kernel trace attributed to kernels by fair share:
every instant at which k kernels run charges 1/k of it to each.  The charges
sum to the time the GPU had any kernel running, so with 8 logical shards
time-sharing one GPU they bound the GPU work per wakeup (a kernel that leaves
the chip partly idle is charged for its share all the same).
usage: python profiles/fair_share.py kernel_trace.csv <skip> <wakeups> [per]"""
import collections
import csv
import sys

path, skip, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
per = int(sys.argv[4]) if len(sys.argv) > 4 else 1
rows = []
for r in csv.DictReader(open(path)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].replace("crgc::", "").replace("void ", "")))
ends = sorted(e for s, e, k in rows if "k_sweep_gather" in k)
t0 = ends[skip * per - 1] if skip else min(s for s, _, _ in rows)
t1 = ends[(skip + n) * per - 1]
ev = []
for s, e, k in rows:
    if s >= t0 and e <= t1 and e > s:
        ev.append((s, 1, k))
        ev.append((e, -1, k))
ev.sort(key=lambda x: (x[0], x[1]))
run = collections.Counter()
share = collections.defaultdict(float)
calls = collections.Counter(k for _, d, k in ev if d == 1)
last = None
for t, d, k in ev:
    if last is not None and run:
        tot = sum(run.values())
        for name, c in run.items():
            share[name] += (t - last) * c / tot
    last = t
    run[k] += d
    if run[k] == 0:
        del run[k]
busy = sum(share.values())
print(f"window {(t1 - t0) / 1e6 / n:.3f} ms per wakeup; busy {busy / 1e6 / n:.3f} ms (fair-share charges below)")
for name, v in sorted(share.items(), key=lambda x: -x[1])[:30]:
    print(f"{v / 1e6 / n:9.3f} ms  {calls[name] / n:8.1f} calls  {name[:80]}")
