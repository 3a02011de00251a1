"""DeltaGraph kernels of a rocprofv3 sqlite kernel trace: per-kernel averages and
the timeline of the last crgc_build_delta_graphs call (from its k_dg_span).
usage: python profiles/dg_kernels.py <run_results.db>"""
import collections
import sqlite3
import sys

rows = sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start").fetchall()
agg = collections.defaultdict(list)
for n, s, e in rows:
    agg[n.split("(")[0]].append(e - s)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    if "dg" in k:
        print(f"{k:40s} n={len(v):4d} avg={sum(v) / len(v) / 1e3:8.1f} us")
idx = [i for i, (n, s, e) in enumerate(rows) if "k_dg_span" in n]
seq = rows[idx[-1]:]
end = next(i for i, (n, s, e) in enumerate(seq) if "k_dg_offsets" in n)
t0 = prev = seq[0][1]
for n, s, e in seq[:end + 1]:
    print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:7.1f} {n.split('(')[0][:40]}")
    prev = e
print(f"span {(prev - t0) / 1e3:.1f} us")
