"""Counter calibration (tools/calib_pmc.hip): FETCH_SIZE / WRITE_SIZE against known bytes.

usage: python profiles/calib_summary.py <calib.jsonl> <fetch counter_collection.csv>
                                         <write counter_collection.csv> <kernel_trace.csv>

For each calibration kernel (its measured launch: the second of the two), prints
the algorithmic bytes, FETCH_SIZE and WRITE_SIZE in bytes (rocprofv3 reports
KiB), the counter-to-byte ratios, bytes per access as the counters see them, and
the kernel-trace duration.  Writes the same as JSON on the last line: the
factors bench.py / pmc_summary.py apply to the trace kernels' counter readings.
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter=None):
    out = collections.defaultdict(list)
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if counter is None:
            out[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        elif r["Counter_Name"] == counter:
            out[k].append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    cal = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")]
    fetch = per_kernel(sys.argv[2], "FETCH_SIZE")
    write = per_kernel(sys.argv[3], "WRITE_SIZE")
    kt = per_kernel(sys.argv[4])
    res = {}
    print(f"{'kernel':16s} {'alg bytes':>13s} {'FETCH':>13s} {'F/alg':>7s} {'WRITE':>13s} {'W/alg':>7s} "
          f"{'F B/acc':>8s} {'ms(kt)':>8s} {'GB/s alg':>9s}")
    for c in cal:
        name = c["kernel"]
        base = name.split("<")[0]
        # template-free names: the two k_rand1 launches come in program order
        def pick(d):
            xs = d.get(base, [])
            if base == "k_rand1":
                which = 0 if "mall" in name else 1
                xs = xs[2 * which: 2 * which + 2]
            return xs[-1] if xs else None
        f, w, t = pick(fetch), pick(write), pick(kt)
        alg = c["algorithmic_bytes"]
        res[name] = {"algorithmic_bytes": alg, "accesses": c["accesses"], "fetch_bytes": f, "write_bytes": w,
                     "fetch_over_alg": f / alg if f else None, "write_over_alg": w / alg if w else None,
                     "fetch_bytes_per_access": f / c["accesses"] if f else None,
                     "ms_kernel_trace": t, "ms_events": c["ms"],
                     "alg_gbs": alg / (t * 1e-3) / 1e9 if t else None}
        r = res[name]
        fmt = lambda x, p=".0f": format(x, p) if x is not None else "-"  # noqa: E731
        print(f"{name:16s} {alg:13d} {fmt(f):>13s} {fmt(r['fetch_over_alg'], '.3f'):>7s} {fmt(w):>13s} "
              f"{fmt(r['write_over_alg'], '.3f'):>7s} {fmt(r['fetch_bytes_per_access'], '.1f'):>8s} "
              f"{fmt(t, '.3f'):>8s} {fmt(r['alg_gbs'], '.0f'):>9s}")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
