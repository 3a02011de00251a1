"""Per-kernel HBM traffic from rocprofv3 --pmc counter_collection CSVs.

usage: python profiles/pmc_summary.py <counter_collection.csv> [more.csv ...]

Prints, per kernel, launches and the mean FETCH_SIZE / WRITE_SIZE per launch
in bytes.  rocprofv3 reports both in KiB.  FETCH_SIZE is also printed doubled:
on gfx950 it tallies 64 B per 128-B request of a wide streaming read
(MI355X_MICROARCH.md, HBM section); other access widths are uncalibrated, so
the raw and doubled values bracket the read bytes of a mixed kernel.
"""
import collections
import csv
import json
import sys


def load(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("crgc::", "")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main():
    agg = load(sys.argv[1:])
    out = {}
    print(f"{'kernel':40s} {'launches':>8s} {'FETCH B/launch':>15s} {'x2':>15s} {'WRITE B/launch':>15s}")
    for k, cs in sorted(agg.items()):
        f = cs.get("FETCH_SIZE", [])
        w = cs.get("WRITE_SIZE", [])
        n = max(len(f), len(w))
        fm = sum(f) / len(f) if f else None
        wm = sum(w) / len(w) if w else None
        out[k] = {"launches": n, "fetch_bytes": fm, "fetch_bytes_x2": 2 * fm if fm is not None else None,
                  "write_bytes": wm}
        fs = f"{fm:15.0f} {2 * fm:15.0f}" if fm is not None else f"{'-':>15s} {'-':>15s}"
        ws = f"{wm:15.0f}" if wm is not None else f"{'-':>15s}"
        print(f"{k[:40]:40s} {n:8d} {fs} {ws}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
