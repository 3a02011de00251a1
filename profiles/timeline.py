"""Timeline of the last wakeup in a rocprofv3 kernel trace: start offset, the
idle gap before each kernel, its duration.  usage: python profiles/timeline.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_ids" in r["Kernel_Name"]]
seq = rows[idx[-2]:idx[-1]]
t0 = int(seq[0]["Start_Timestamp"])
prev = t0
busy = 0
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("crgc::", "")[:30]
    q = r.get("Queue_Id", "?")
    print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:7.1f} dur {(e - s) / 1e3:7.1f} q{q} {name}")
    busy += e - s
    prev = max(prev, e)
print(f"span {(prev - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")
