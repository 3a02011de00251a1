"""Garbage-set parity at the sizes the bench numbers are quoted on.

The checker is the OpenMP engine (oracle/omp_graph.cpp): its garbage and kill
sets, live / pseudo-root / traced-edge counts are pinned to the single-thread
oracle's by tests/test_omp_graph_cpu.py, and it finishes a 1e8-edge wakeup in
a fraction of a second on the box's cores where the oracle would take minutes.

  * C2 at full size, the bench's own stream (bench.py: seed 0x5EED + 2,
    location 1, 1e7 actors / 1e8 edges, 1e6-entry wakeups with 9 % busy and
    1 % in flight): every trace compared, sets and counts.
  * C5 at full size (8 nodes x 1.25e6 actors: node 1's entries, the other
    nodes' DeltaGraphs and UndoLog folds, a downed node's replay).
  * C4's construction (8 producers of one node, workload/world.py
    c4_producer) at 2.5e7 actors / 2.5e8 edges — a quarter of C4 (VERDICT
    r5 #6; a tenth until round 5) — on G = 8 logical shards of one MI355X
    (the 8-GPU layout; in-process transport), against the unsharded OpenMP
    engine, two §8d wakeups.

Reference semantics: ShadowGraph.java:205-289 (trace), :75-125 (mergeEntry),
:127-174 (mergeDelta, mergeUndoLog).
"""
import os

import numpy as np
import pytest

import world

pytestmark = pytest.mark.gpu

THREADS = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))


def _same(rh, ro, what):
    assert rh.n_live == ro["live"], what
    assert rh.pseudo_roots == ro["pseudo_roots"], what
    assert rh.edges_scanned == ro["edges_scanned"], what
    assert len(rh.garbage) == ro["garbage"] and len(rh.kill) == ro["kill"], what
    assert np.array_equal(np.sort(rh.garbage), np.sort(ro["garbage_ids"])), what
    assert np.array_equal(np.sort(rh.kill), np.sort(ro["kill_ids"])), what


def test_c2_full_size_garbage_sets_match_openmp(hip_mod, oracle_mod):
    V, E, B = 10_000_000, 100_000_000, 1_000_000
    w = world.World(seed=0x5EED + 2, location=1)      # bench.py's rank-0 C2 node
    w.bulk_graph(V, E, alpha=2.1, n_roots=V // 1000, cap=100000)
    h = hip_mod.ShadowGraph(vertex_capacity=int(V * 1.2), edge_capacity=int(E * 1.2))
    p = oracle_mod.OmpGraph(threads=THREADS, vertex_hint=int(V * 1.5))
    p.reserve_ids(1 << 20)
    for b in w.batches(1 << 20):
        h.merge_entries(b.to_device())
        p.merge_entries(b)
    rh, rp = h.trace(True), p.trace(True, ids=True)
    _same(rh, rp, "after the load")
    assert rh.n_live > 0.99 * V
    for k in range(2):
        b = w.wakeup(B, busy=V * 9 // 100, pending=V // 100)
        h.merge_entries(b.to_device())
        p.merge_entries(b)
        rh, rp = h.trace(True), p.trace(True, ids=True)
        _same(rh, rp, f"wakeup {k}")
        assert rh.pseudo_roots > 0.07 * rh.n_live          # the §8d cut: ~10 % busy / in flight
        assert rh.edges_scanned > 0.9 * E
        assert len(rh.garbage) > 0 and len(rh.kill) > 0


@pytest.mark.timeout(600)
def test_c4_construction_eight_logical_shards_match_openmp(hip_mod, oracle_mod):
    import math
    V, E = 25_000_000, 250_000_000                     # C4's construction at 1/4 scale
    P = world.C4_PRODUCERS
    ws = [world.c4_producer(k, V // P, E // P) for k in range(P)]
    far = V * (1.0 - math.exp(-E / (8 * V)))            # proxies per shard (bench.py capacity_hints)
    h = hip_mod.ShardedShadowGraph(8, vertex_capacity=int(V / 8 * 1.1), edge_capacity=int(E / 8 * 1.15),
                                   proxy_capacity=int(far * 1.05))
    p = oracle_mod.OmpGraph(threads=THREADS, vertex_hint=int(V * 1.5))
    p.reserve_ids(V // 8)  # (the planted dead components: ~5 % of the actors at the first trace)
    try:
        for w in ws:
            for b in w.batches(1 << 20):
                h.merge_entries(b, split=True)          # every shard contributes a part
                p.merge_entries(b)
        rh, rp = h.trace(True), p.trace(True, ids=True)
        _same(rh, rp, "after the load")
        for k in range(2):
            from crgc_hip.batch import EntryBatch
            b = EntryBatch.concat([w.wakeup(V // 10 // P, busy=V // P * 9 // 100, pending=V // P // 100)
                                   for w in ws])
            h.merge_entries(b, split=True)
            p.merge_entries(b)
            rh, rp = h.trace(True), p.trace(True, ids=True)
            _same(rh, rp, f"wakeup {k}")
            assert rh.rounds >= 2 and rh.ids_sent > 0      # marks crossed shards
            assert rh.pseudo_roots > 0.07 * rh.n_live
        assert h.total_actors_seen() >= V
    finally:
        h.close()


@pytest.mark.timeout(400)
def test_c5_full_size_cluster_stream_and_downed_node_match_openmp(hip_mod, oracle_mod):
    """C5 exactly as `bench.py --workload c5` builds it, at full size (VERDICT
    r5 #6; tests/test_hip_bench_size.py keeps the 1/10 form with the UndoLog
    folds checked field by field): 8 simulated nodes of 1.25e6 actors / 1.25e7
    edges; node 1 merges its own entries and the other seven nodes'
    DeltaGraphs (LocalGC.scala:124-136), 1.25e5-entry wakeups per node, and
    folds every remote node's deltas into its UndoLog on the device; then node
    8 is downed and its log replayed (ShadowGraph.mergeUndoLog,
    :158-174).  The checker is the OpenMP engine, whose mergeDelta /
    mergeUndoLog are pinned to the oracle by tests/test_omp_graph_cpu.py."""
    from crgc_hip import DeltaBatch, abi
    from test_hip_undo_acc import _canon
    nodes, V, E, B = 8, 1_250_000, 12_500_000, 125_000
    ws = [world.World(seed=0x5EED + 5 + 1000 * k, location=k + 1) for k in range(nodes)]
    for w in ws:
        w.bulk_graph(V, E, alpha=2.1, n_roots=max(1, V // 1000), cap=100000)
    h = hip_mod.ShadowGraph(vertex_capacity=int(nodes * V * 1.2), edge_capacity=int(nodes * E * 1.2))
    p = oracle_mod.OmpGraph(threads=THREADS, vertex_hint=int(nodes * V * 1.5))
    p.reserve_ids(nodes * V)  # the downed node's trace reports up to all its shadows
    accs = [h.undo_accumulator(k + 1) for k in range(1, nodes)]
    for k, w in enumerate(ws):
        for b in w.batches(1 << 20):
            if k == 0:
                h.merge_entries(b.to_device())
                p.merge_entries(b)
            else:
                d = world.deltas_of(b)[0]
                dd = d.to_device()
                h.merge_deltas(dd)
                p.merge_deltas(d)
                accs[k - 1].fold_deltas(dd)
    rh, rp = h.trace(True), p.trace(True, ids=True)
    _same(rh, rp, "after the load")
    assert rh.n_live > 0.9 * nodes * V

    def wakeup():
        own = ws[0].wakeup_batch(B)
        parts = [world.deltas_of(ws[k].wakeup_batch(B))[0] for k in range(1, nodes)]
        deltas = DeltaBatch.concat(parts)
        h.merge_deltas(deltas.to_device())
        h.merge_entries(own.to_device())
        p.merge_deltas(deltas)
        p.merge_entries(own)
        return parts

    for k in range(2):
        parts = wakeup()
        for acc, part in zip(accs, parts):
            acc.fold_deltas(part.to_device())
        rh, rp = h.trace(True), p.trace(True, ids=True)
        _same(rh, rp, f"wakeup {k}")
        assert rh.pseudo_roots > 0 and rh.edges_scanned > 0.5 * nodes * E
    assert h.total_actors_seen() >= nodes * V
    # node 8 is downed: its deltas since the last trace are undone, then trace
    parts = wakeup()
    last8 = h.undo_accumulator(nodes)
    last8.fold_deltas(parts[-1].to_device())
    log = world.undo_of(parts[-1], nodes)
    assert _canon(last8.export()) == _canon(log)
    try:
        p.merge_undo(log)
        cme = None
    except abi.CrgcError as e:
        cme = e.code
    if cme is None:
        h.merge_undo_acc(last8)
        rh, rp = h.trace(True), p.trace(True, ids=True)
        _same(rh, rp, "node 8 downed")
    else:
        with pytest.raises(abi.CrgcError) as e:
            h.merge_undo_acc(last8)
        assert e.value.code == cme
