"""One shard of a hash-partitioned shadow graph in its own process (rank r of
torch.distributed over gloo), the shards exchanging through the product's host
transport (crgc_transport_host, staging in pinned host memory) — the protocol
of one process per GPU with a host collective in place of RCCL, which refuses
two ranks on one GPU.  Run by tests/test_hip_multiprocess.py, two or three
ranks on the test box's one MI355X.  Rank 0 also replays the same stream into
the unsharded oracle and checks every wakeup's garbage / kill sets, live count,
pseudo-roots and traced edges against the union of the ranks' results.

usage: python tests/mp_shard_worker.py <rank> <world> <port> <out.json>
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, "uigc-akka_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "workload"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    rank, world_size, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = port
    import numpy as np
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    import crgc_hip
    import world
    coll = crgc_hip.HostCollectives(world_size, rank)
    tr = crgc_hip.Transport.host(coll, device=0)
    g = crgc_hip.ShadowGraph(device=0, n_shards=world_size, shard=rank, transport=tr)
    o = None
    if rank == 0:
        import oracle
        o = oracle.OracleGraph()
    w = world.World(seed=0x5EED + 21)
    V = 20_000
    w.bulk_graph(V, 10 * V, alpha=2.1, n_roots=V // 1000, cap=10000)
    batches = list(w.batches(1 << 16))
    checks = []

    def step(b):
        g.merge_entries(b.split(world_size)[rank])  # this rank contributes its part of the batch
        if o is not None:
            o.merge_entries(b)
        r = g.trace(True)
        mine = {"garbage": sorted(int(x) for x in r.garbage), "kill": sorted(int(x) for x in r.kill),
                "n_live": int(r.n_live), "pseudo_roots": int(r.pseudo_roots),
                "edges_scanned": int(r.edges_scanned), "rounds": int(r.rounds)}
        allr = [None] * world_size
        dist.all_gather_object(allr, mine)
        if o is not None:
            ro = o.trace(True)
            union_g = sorted(x for a in allr for x in a["garbage"])
            union_k = sorted(x for a in allr for x in a["kill"])
            checks.append({
                "garbage": union_g == sorted(int(x) for x in ro.garbage),
                "kill": union_k == sorted(int(x) for x in ro.kill),
                "n_live": sum(a["n_live"] for a in allr) == int(ro.n_live),
                "pseudo_roots": sum(a["pseudo_roots"] for a in allr) == int(ro.pseudo_roots),
                "edges_scanned": sum(a["edges_scanned"] for a in allr) == int(ro.edges_scanned),
                "rounds": max(a["rounds"] for a in allr), "n_garbage": len(union_g)})

    for b in batches:
        step(b)
    for _ in range(3):
        step(w.wakeup(V // 10, busy=V * 9 // 100, pending=V // 100))
    g.close()
    tr.close()
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"checks": checks, "identical": all(c["garbage"] and c["kill"] and c["n_live"]
                                                          and c["pseudo_roots"] and c["edges_scanned"]
                                                          for c in checks)}, f)


if __name__ == "__main__":
    main()
