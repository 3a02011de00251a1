"""Summarise a rocprofv3 kernel trace: steady-state per-kernel time per wakeup.

usage: python profiles/summarize.py <run_kernel_trace.csv> [n_steps]
Takes the last n_steps wakeups (each starts at a k_ids launch).
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_ids" in r["Kernel_Name"]]
start = idx[-n]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[start:]:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':48s} {'calls/step':>10s} {'us/step':>9s} {'avg_us':>8s}")
for k, (c, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k[:48]:48s} {c / n:10.1f} {us / n:9.1f} {us / c:8.1f}")
print(f"{'total device time per wakeup (us)':48s} {'':10s} {tot / n:9.1f}")
one = [r for r in rows[idx[-1]:]]
seq = [(r["Kernel_Name"].split("(")[0].replace("void crgc::", "")[:22],
        round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1)) for r in one]
print("last wakeup kernel sequence:", seq)
