"""Bytes a sharded mark exchanges per wakeup in each form (CRGC_XBITS 0 / 1 / 2)
on a C4-shaped graph: G logical shards on one GPU (in-process transport)."""
import json
import os

os.environ.setdefault("CRGC_TEST_HOOKS", "1")  # the variants are test hooks (crgc_api.hip Knobs)
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "uigc-akka_amd"), os.path.join(ROOT, "workload")]
import crgc_hip  # noqa: E402
import world  # noqa: E402

G = int(os.environ.get("XG", "8"))
V = int(os.environ.get("XV", "1000000"))
out = {"G": G, "actors": V, "edges": 10 * V, "forms": {}}
for xb in ("0", "1", "2"):
    os.environ["CRGC_XBITS"] = xb
    w = world.World(seed=0x5EED + 4)
    w.bulk_graph(V, 10 * V, alpha=2.1, n_roots=V // 1000, cap=100000)
    h = crgc_hip.ShardedShadowGraph(G, vertex_capacity=int(V * 2.0), edge_capacity=int(12 * V))
    for b in w.batches(1 << 20):
        h.merge_entries(b, split=True)
    h.trace(True)
    recs = []
    for _ in range(4):
        b = w.wakeup(V // 10, busy=V * 9 // 100, pending=V // 100)
        h.merge_entries(b, split=True)
        t = time.perf_counter()
        r = h.trace(True)
        recs.append((time.perf_counter() - t, r))
    h.close()
    last = recs[1:]
    out["forms"][xb] = {
        "rounds": [r.rounds for _, r in last],
        "marks_sent": sum(r.ids_sent for _, r in last) / len(last),
        "exchange_bytes": sum(r.exchange_bytes for _, r in last) / len(last),
        "ms_exchange": sum(r.ms_exchange for _, r in last) / len(last),
        "ms_trace_wall": 1e3 * sum(t for t, _ in last) / len(last),
    }
    print(json.dumps({xb: out["forms"][xb]}), file=sys.stderr, flush=True)
print(json.dumps(out))
