"""Interleaved A/B timing of trace variants on one resident C2 graph.

Variants are selected by environment switches read per trace (CRGC_* in
crgc_api.hip); results must be identical, only timings differ.

    python tools/ab_trace.py --actors 10000000 --edges 100000000 --rounds 8 \
        --variant CRGC_PULL=0 --variant CRGC_PULL=1,CRGC_PULL_DIV=32
"""
import argparse
import json
import os

os.environ.setdefault("CRGC_TEST_HOOKS", "1")  # the variants are test hooks (crgc_api.hip Knobs)
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uigc-akka_amd", "workload", ""):
    sys.path.insert(0, os.path.join(REPO, sub))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--actors", type=int, default=10_000_000)
    ap.add_argument("--edges", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--wakeups", type=int, default=3, help="bench wakeups applied before timing")
    ap.add_argument("--variant", action="append", default=[])
    args = ap.parse_args()
    import torch
    import crgc_hip
    import world
    import bench
    ns = argparse.Namespace(actors=args.actors, edges=args.edges, batch=1_000_000, workload="c2")
    stream = torch.cuda.Stream()
    w, g = bench.build_graph(crgc_hip, world, 0, 0, stream.cuda_stream, ns)  # bench's C2 graph
    for _ in range(args.wakeups):
        b = bench.wakeup_batches(w, ns, 1)[0].to_device("cuda")
        torch.cuda.synchronize()  # uploaded on torch's stream, merged on the graph's
        g.merge_entries(b)
        g.trace_counts(True)
    variants = args.variant or ["BASE=0"]
    res = {v: [] for v in variants}
    ref = None
    shape = {}
    for r in range(args.rounds):
        for v in variants:
            kv = [x.split("=") for x in v.split(",")]
            for k, val in kv:
                os.environ[k] = val
            t = time.perf_counter()
            out, ng, nk = g.trace_counts(True)
            wall = (time.perf_counter() - t) * 1e3
            # levels / edges_scanned depend on the direction and k_tail switches;
            # the live set and the garbage count may not
            key = (out.n_live, ng, nk)
            ref = ref or key
            assert key == ref, (v, key, ref)
            shape.setdefault(v, (out.edges_scanned, out.levels))
            res[v].append((out.ms_mark, out.ms_sweep, wall))
            for k, _ in kv:
                del os.environ[k]
    summary = {}
    for v, xs in res.items():
        summary[v] = {"mark_ms_median": statistics.median(x[0] for x in xs),
                      "mark_ms_min": min(x[0] for x in xs),
                      "sweep_ms_median": statistics.median(x[1] for x in xs),
                      "wall_ms_median": statistics.median(x[2] for x in xs),
                      "edges_scanned": shape[v][0], "levels": shape[v][1]}
    print(json.dumps({"shape": {"live": ref[0], "garbage": ref[1], "kill": ref[2]},
                      "variants": summary}))


if __name__ == "__main__":
    main()
