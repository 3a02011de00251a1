"""The C++ C5 stream builders (workload/deltas.cpp, world.undo_of) against the
Python restatements of DeltaGraph / UndoLog (workload/delta.py), on CPU."""
import numpy as np

import delta
import world
from crgc_hip import DeltaBatch

FIELDS = ("id", "recv_count", "supervisor", "flags", "out_off", "out_target", "out_count")


def _batches():
    w = world.World(seed=3, location=2)
    w.bulk_graph(3000, 30000, alpha=2.1, n_roots=30)
    yield w.take(20000)            # spawn tree + acquaintance edges
    yield w.wakeup_batch(5000)     # sends, shares, releases, receives


def test_cpp_delta_builder_matches_python_restatement():
    for b in _batches():
        d, graph_off = world.deltas_of(b)
        gs = delta.deltas_from_entries(b.to_entries(), address=2)
        ref = DeltaBatch.concat([g.to_batch() for g in gs])
        assert len(graph_off) - 1 == len(gs)
        assert list(np.diff(graph_off)) == [g.size for g in gs]
        for k in FIELDS:
            assert np.array_equal(getattr(d, k), getattr(ref, k)), k


def _canon(u):
    out = {}
    for i, a in enumerate(u.actor.tolist()):
        refs = {int(t): int(c) for t, c in zip(u.created_target[u.created_off[i]:u.created_off[i + 1]],
                                               u.created_count[u.created_off[i]:u.created_off[i + 1]])}
        out[a] = (int(u.message_count[i]), refs)
    return out


def test_undo_of_matches_python_undo_log():
    for b in _batches():
        d, _ = world.deltas_of(b)
        log = delta.UndoLog(2)
        for g in delta.deltas_from_entries(b.to_entries(), address=2):
            log.mergeDeltaGraph(g)
        assert _canon(world.undo_of(d, 2)) == _canon(log.to_batch())


def test_c1_generator_has_the_stated_shape(oracle_mod):
    """C1 (BASELINE.json config 1): ~1e6 refs over 1e5 actors, counts
    1 / 2 / -1 at 90 / 8 / 2 %, 5 % dead components, and at every wakeup ~1 %
    roots + 9 % busy + 1 % with mail in flight."""
    from collections import Counter
    V = 100_000
    w = world.World(seed=0x5EED + 1)
    w.set_mix(send=0.2, share=0.2, release=0.2, spawn=0.2, actions_per_msg=2.0)
    w.uniform_graph(V, mean_acq=8.0, n_roots=V // 100, dead_frac=0.05)
    o = oracle_mod.OracleGraph()
    for b in w.batches(1 << 20):
        o.merge_entries(b)
    st = o.export()
    n_edges = len(st.edges)
    assert 0.9e6 < n_edges < 1.2e6
    acq = Counter(c for (a, t), c in st.edges.items() if a != t)
    tot = sum(acq.values())
    assert acq[-1] / tot > 0.01 and acq[2] / tot > 0.05 and acq[1] / tot > 0.85
    r = o.trace(True)
    assert len(r.garbage) == V // 20 and len(r.kill) == V // 20
    for _ in range(3):
        o.merge_entries(w.wakeup(10_000, busy=V * 9 // 100, pending=V // 100))
        r = o.trace(True)
    assert w.n_busy() == V * 9 // 100
    assert 0.09 * r.n_live < r.pseudo_roots < 0.13 * r.n_live


def test_c4_producers_share_no_id_and_concat_keeps_queue_order(oracle_mod):
    """C4 is one node's graph from 8 producers (workload/world.py c4_producer):
    their id spaces are disjoint, and EntryBatch.concat of their wakeup parts
    merges exactly like the parts one after the other (offsets rebased)."""
    from crgc_hip import EntryBatch
    ws = [world.c4_producer(k, 4000, 40000) for k in range(world.C4_PRODUCERS)]
    seen = set()
    for w in ws:
        ids = set()
        for b in w.batches(1 << 20):
            ids |= set(b.self.tolist()) | set(b.created_target.tolist())
        assert not (ids & seen)
        seen |= ids
        assert all((i >> 48) == 1 for i in ids)      # one node: location 1
    parts = [w.wakeup(400, busy=360, pending=40) for w in ws]
    cat = EntryBatch.concat(parts)
    assert cat.n_entries == sum(p.n_entries for p in parts)
    a, b = oracle_mod.OracleGraph(), oracle_mod.OracleGraph()
    a.merge_entries(cat)
    for p in parts:
        b.merge_entries(p)
    assert a.export() == b.export()
