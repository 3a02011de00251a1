"""Per-kernel HBM traffic from rocprofv3 --pmc counter_collection CSVs.

usage: python profiles/pmc_summary.py [--last-wakeups N] [--fetch-factor X] <csv> [more.csv ...]

Prints, per kernel, launches and the mean FETCH_SIZE / WRITE_SIZE per launch in
bytes (rocprofv3 reports KiB).  --last-wakeups N keeps only the dispatches of the
last N wakeups of a bench run (each starts at a k_ids dispatch), i.e. steady
state, not the graph's bulk load.  --fetch-factor X scales FETCH_SIZE by the
calibration factor of the kernel's own access shapes (profiles/calib_summary.py);
the default 1 reports the raw counter.
"""
import argparse
import collections
import csv
import json


def load(paths, last_wakeups):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        rows = list(csv.DictReader(open(p)))
        rows.sort(key=lambda r: int(r.get("Dispatch_Id") or 0))
        if last_wakeups:
            starts = [i for i, r in enumerate(rows) if "k_ids" in r["Kernel_Name"]]
            starts = sorted(set(int(rows[i]["Dispatch_Id"]) for i in starts))
            if len(starts) >= last_wakeups:
                first = starts[-last_wakeups]
                rows = [r for r in rows if int(r["Dispatch_Id"]) >= first]
        for r in rows:
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("crgc::", "")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--last-wakeups", type=int, default=0)
    ap.add_argument("--fetch-factor", type=float, default=1.0)
    ap.add_argument("csv", nargs="+")
    a = ap.parse_args()
    agg = load(a.csv, a.last_wakeups)
    out = {}
    print(f"{'kernel':40s} {'launches':>8s} {'FETCH B/launch':>15s} {'WRITE B/launch':>15s}")
    for k, cs in sorted(agg.items()):
        f = cs.get("FETCH_SIZE", [])
        w = cs.get("WRITE_SIZE", [])
        n = max(len(f), len(w))
        fm = sum(f) / len(f) if f else None
        wm = sum(w) / len(w) if w else None
        out[k] = {"launches": n, "fetch_bytes": fm, "write_bytes": wm,
                  "fetch_bytes_calibrated": fm * a.fetch_factor if fm is not None else None}
        fs = f"{fm:15.0f}" if fm is not None else f"{'-':>15s}"
        ws = f"{wm:15.0f}" if wm is not None else f"{'-':>15s}"
        print(f"{k[:40]:40s} {n:8d} {fs} {ws}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
