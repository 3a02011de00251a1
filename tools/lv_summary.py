"""Per-level kernel times of a CRGC_LEVEL_LOG=1 CRGC_KERNEL_TIMING=2 run, averaged
over the last N traces: level, frontier size, k_frontier / k_tail / k_expand us.
usage: python3 tools/lv_summary.py <levels.err> [N]"""
import re
import sys

pat = re.compile(r"\[crgc\] level (\d+) frontier (\d+)\s+([\d.]+) us \(frontier ([\d.]+) tail ([\d.]+) expand ([\d.]+)\)")
traces = []
for line in open(sys.argv[1]):
    m = pat.search(line)
    if not m:
        continue
    lv = int(m.group(1))
    if lv == 0:
        traces.append([])
    if traces:
        traces[-1].append([float(x) for x in m.groups()])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
last = traces[-n:]
depth = max(len(t) for t in last)
tot = [0.0, 0.0, 0.0]
for lv in range(depth):
    rows = [t[lv] for t in last if len(t) > lv]
    avg = [sum(r[k] for r in rows) / len(rows) for k in range(6)]
    for k in range(3):
        tot[k] += avg[3 + k]
    print(f"L{lv:<3d} front {avg[1]:>11.0f}  frontier {avg[3]:7.1f}  tail {avg[4]:6.1f}  expand {avg[5]:7.1f}")
print(f"sum  frontier {tot[0]:.1f}  tail {tot[1]:.1f}  expand {tot[2]:.1f}  all {sum(tot):.1f} us per trace (last {len(last)})")
