"""Kernel time per wakeup from a rocprofv3 kernel_trace.csv: dispatches after the
`skip`-th wakeup's last k_sweep_gather, grouped by kernel, divided by the
wakeups in the window (`per` k_sweep_gathers make one wakeup: the shard count of
a --logical-shards run, 1 otherwise).
usage: python profiles/wakeup_kernels.py kernel_trace.csv <skip> <wakeups> [per]"""
import collections
import csv
import sys

path, skip, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
per = int(sys.argv[4]) if len(sys.argv) > 4 else 1
rows = []
for r in csv.DictReader(open(path)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
ends = [e for s, e, k in rows if "k_sweep_gather" in k]
t0 = ends[skip * per - 1] if skip else rows[0][0]
t1 = ends[(skip + n) * per - 1]
agg = collections.defaultdict(lambda: [0, 0])
for s, e, k in rows:
    if s >= t0 and e <= t1:
        name = k.split("(")[0].replace("crgc::", "").replace("void ", "")
        agg[name][0] += 1
        agg[name][1] += e - s
tot = sum(v[1] for v in agg.values())
print(f"window {(t1 - t0) / 1e6 / n:.3f} ms per wakeup; kernel time {tot / 1e6 / n:.3f} ms per wakeup "
      f"(summed over concurrent streams)")
for name, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
    print(f"{d / 1e6 / n:9.3f} ms  {c / n:8.1f} calls  {d / c / 1e3:9.1f} us avg  {name[:80]}")
