"""N > 1 host paths on CPU ranks (torch.distributed, gloo backend, 127.0.0.1).

* The sharded trace protocol (tests/shard_model.py: local fixpoints, marked
  proxies exchanged per round, remote kill requests) reproduces the unsharded
  oracle's garbage / kill sets and live count on world_size 2 and 3, wakeup by
  wakeup, on seeded adversarial streams (tests/fuzz.py).
* bench.py's distributed plumbing: the stats reduction (sum / max over ranks)
  that turns per-rank numbers into the whole-job value.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    for sub in ("uigc-akka_amd", "workload", "oracle", "tests"):
        sys.path.insert(0, os.path.join(REPO, sub))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _protocol_worker(rank, world, port, seed, q):
    dist = _init(rank, world, port)
    try:
        import fuzz
        import oracle
        from shard_model import ShardModel
        o = oracle.OracleGraph()
        fz = fuzz.Fuzz(seed)
        checked = 0
        for step in range(10):
            eb = fz.entries(150 + 40 * step)
            o.merge_entries(eb)
            if step % 2:
                o.merge_deltas(fz.deltas(4))
            if step == 6:
                o.merge_undo(fz.undo(o.export().vertices.keys()))
            state = o.export()
            g, k, live, rounds = ShardModel(state, rank, world).trace(dist)
            parts = [None] * world
            dist.all_gather_object(parts, (sorted(g), sorted(k), live))
            ro = o.trace(True)
            if rank == 0:
                G = set().union(*(set(p[0]) for p in parts))
                K = set().union(*(set(p[1]) for p in parts))
                assert sum(len(p[0]) for p in parts) == len(G)  # homes partition the ids
                assert G == ro.garbage_set(), step
                assert K == ro.kill_set(), step
                assert sum(p[2] for p in parts) == ro.n_live, step
            checked += 1
            fz.sync(o.export())
        q.put((rank, "ok", checked))
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put((rank, "error", traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _run(worker, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, status, info in out:
        assert status == "ok", f"rank {rank}: {info}"
    return out


@pytest.fixture(scope="module", autouse=True)
def _built():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    oracle.build()
    from crgc_hip import abi
    abi.load_library()  # crgc_shard_of is a pure host function


@pytest.mark.parametrize("world,seed", [(2, 31), (3, 32)])
def test_sharded_protocol_matches_oracle_over_gloo(world, seed):
    out = _run(_protocol_worker, world, seed)
    assert all(c == 10 for _, _, c in out)


def _stats_worker(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        import torch
        # what bench.py reduces: (edges, entries, wall, ...) summed and max'ed
        stats = torch.tensor([100.0 * (rank + 1), 10.0, 1.0 + rank], dtype=torch.float64)
        tot, mx = stats.clone(), stats.clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        value = tot[0].item() / mx[2].item()
        expect = sum(100.0 * (r + 1) for r in range(world)) / (1.0 + world - 1)
        assert abs(value - expect) < 1e-9
        q.put((rank, "ok", value))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_bench_whole_job_value_reduction_over_gloo():
    _run(_stats_worker, 2)
