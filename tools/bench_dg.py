"""Timing of crgc_build_delta_graphs on C2-mix wakeup batches (host / device
outputs), for profiling:  python tools/bench_dg.py [--entries N] [--reps K]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uigc-akka_amd", "workload"):
    sys.path.insert(0, os.path.join(REPO, sub))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--entries", type=int, nargs="+", default=[125_000, 1_000_000])
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import crgc_hip
    import world
    g = crgc_hip.ShadowGraph()
    w = world.World(seed=0x5EED + 9, location=1)
    w.bulk_graph(1_000_000, 10_000_000, alpha=2.1, n_roots=1000)
    w.take(w.queued())
    out = {}
    for n in args.entries:
        b = w.wakeup_batch(n).to_device()
        torch.cuda.synchronize()
        for dev_out in (False, True):
            g.build_delta_graphs(b, device_out=dev_out)  # warm: buffers sized
            ts = []
            for _ in range(args.reps):
                t = time.perf_counter()
                _, goff, _, _ = g.build_delta_graphs(b, device_out=dev_out)
                ts.append(time.perf_counter() - t)
            out[f"{n}_{'device' if dev_out else 'host'}"] = {
                "graphs": int(len(goff) - 1), "ms_min": min(ts) * 1e3,
                "entries_per_s": n / min(ts)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
