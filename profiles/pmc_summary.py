"""Per-kernel HBM traffic from rocprofv3 --pmc counter_collection CSVs.

usage: python profiles/pmc_summary.py [--last-wakeups N] [--fetch-factor X] <csv> [more.csv ...]

Prints, per kernel, launches and the mean FETCH_SIZE / WRITE_SIZE per launch in
bytes (rocprofv3 reports KiB).  --last-wakeups N keeps only the dispatches of the
last N wakeups of a bench run (each starts at a k_ids dispatch), i.e. steady
state, not the graph's bulk load.  --fetch-factor X scales FETCH_SIZE by the
calibration factor of the kernel's own access shapes (profiles/calib_summary.py);
the default 1 reports the raw counter.  --calibrate doubles FETCH_SIZE for the
kernels whose reads are wide streaming loads (STREAMING below): the calibration
kernels read 0.50 x the bytes of 16-B and 8-B/lane streaming reads
(profiles/r2d/calib_summary.txt, /opt/skills/guides/MI355X_MICROARCH.md), while
random 1-B / 4-B accesses count a line each and stay as counted.
"""
import argparse
import collections
import csv
import json


# Kernels whose fetched bytes are (mostly) coalesced 8/16-B per lane streams
# over slot, entry or atom arrays; the rest are dominated by random line
# accesses (id / edge probes, candidate stores), which the counter sees whole.
STREAMING = {
    "k_frontier<true, false>", "k_frontier<true, true>",  # flags / recv / sup per slot
    "k_sweep", "k_sweep_scan", "k_trace_reset",            # per-slot passes
    "k_entries_atoms", "k_ep_count", "k_ep_scatter",        # the batch and atom streams
    "k_scan_sums", "k_scan_apply_top", "k_copy_lists", "k_copy_segs", "k_copy_ranges",
    "k_xscan<false>", "k_xscan<true>",
}


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


def wide_expand(paths, last_wakeups):
    """Bytes per wakeup of the wide levels' expand — level 0 (k_bin_place +
    k_bin_apply) and level 1 (the first k_expand after them) — the launches the
    library times by default (CRGC_KERNEL_TIMING=3): {counter: mean bytes}."""
    out = {}
    for p in paths:
        rows = list(csv.DictReader(open(p)))
        rows.sort(key=lambda r: int(r.get("Dispatch_Id") or 0))
        per = []  # per wakeup (each starts at a k_ids dispatch)
        cur, seen_bin, seen_l1 = None, False, False
        for r in rows:
            k = r["Kernel_Name"]
            if "k_ids" in k:
                cur, seen_bin, seen_l1 = {}, False, False
                per.append(cur)
                continue
            if cur is None:
                continue
            name = r["Counter_Name"]
            if "k_bin_place" in k or "k_bin_apply" in k:
                seen_bin = True
                cur[name] = cur.get(name, 0.0) + float(r["Counter_Value"]) * 1024.0
            elif "k_expand" in k and seen_bin and not seen_l1:
                seen_l1 = True
                cur[name] = cur.get(name, 0.0) + float(r["Counter_Value"]) * 1024.0
        per = [w for w in per if w][-last_wakeups:] if last_wakeups else [w for w in per if w]
        for w in per:
            for n, v in w.items():
                out.setdefault(n, []).append(v)
    return {n: sum(v) / len(v) for n, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--last-wakeups", type=int, default=0)
    ap.add_argument("--fetch-factor", type=float, default=1.0)
    ap.add_argument("--calibrate", action="store_true",
                    help="x2 FETCH_SIZE for the STREAMING kernels (overrides --fetch-factor there)")
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
        ff = 2.0 if a.calibrate and k in STREAMING else a.fetch_factor
        out[k] = {"launches": n, "fetch_bytes": fm, "write_bytes": wm,
                  "fetch_bytes_calibrated": fm * ff if fm is not None else None,
                  "fetch_factor": ff}
        fs = f"{fm:15.0f}" if fm is not None else f"{'-':>15s}"
        ws = f"{wm:15.0f}" if wm is not None else f"{'-':>15s}"
        print(f"{k[:40]:40s} {n:8d} {fs} {ws}")
    wide = wide_expand(a.csv, a.last_wakeups)
    if wide:
        print(f"wide-level expand (levels 0 + 1) per wakeup: {wide}")
        out["_wide_expand_per_wakeup"] = wide
    print(json.dumps(out))


if __name__ == "__main__":
    main()
