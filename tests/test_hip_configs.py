"""HIP vs oracle on the BASELINE.json configurations (C1, C2 scaled, C3, C5).

C1 / C2 wakeups follow SURVEY §8d: about 9 % of the actors busy and 1 % with
mail in flight when LocalGC drains the queue (workload/world.cpp wl_wakeup).

Bit-exact parity is checked on garbage and kill *sets*, live counts and the
exported graph state, wakeup by wakeup, at sizes the oracle finishes in
seconds.  The full-size C2 graph is checked by size-independent properties
(test_c2_full_size_properties).
"""
import numpy as np
import pytest

import cluster
import world

pytestmark = pytest.mark.gpu


def _same(rh, ro):
    assert rh.garbage_set() == ro.garbage_set()
    assert rh.kill_set() == ro.kill_set()
    assert len(rh.garbage) == len(ro.garbage) and len(rh.kill) == len(ro.kill)
    assert rh.n_live == ro.n_live
    assert rh.pseudo_roots == ro.pseudo_roots
    assert rh.sup_edges == ro.sup_edges
    assert rh.edges_scanned == ro.edges_scanned


def _load(g, w, batch):
    for b in w.batches(batch):
        g.merge_entries(b)


def c1_world(actors=100_000, seed=0x5EED + 1):
    """C1 as BASELINE.json / SURVEY §8d state it: 1e5 actors, uniform 1 + Poisson
    acquaintances (~1e6 refs, counts 1 / 2 / -1), 1 % roots, 5 % planted dead
    components, RandomSpec's op mix (RandomSpec.scala:69-87)."""
    w = world.World(seed=seed)
    w.set_mix(send=0.2, share=0.2, release=0.2, spawn=0.2, actions_per_msg=2.0)
    w.uniform_graph(actors, mean_acq=8.0, n_roots=actors // 100, dead_frac=0.05)
    return w


def busy_wakeup(w, actors, batch):
    """A wakeup with 9 % of the actors busy and 1 % with mail in flight at the cut."""
    return w.wakeup(batch, busy=actors * 9 // 100, pending=actors // 100)


def test_c1_spec_wakeups_match_oracle(hip_mod, oracle_mod):
    actors = 100_000
    w = c1_world(actors)
    h = hip_mod.ShadowGraph(vertex_capacity=actors, edge_capacity=10 * actors)
    o = oracle_mod.OracleGraph()
    for b in w.batches(1 << 20):
        h.merge_entries(b)
        o.merge_entries(b)
    r0 = o.trace(True)
    _same(h.trace(True), r0)
    assert len(r0.garbage) == actors // 20            # the planted dead components
    for k in range(6):
        b = busy_wakeup(w, actors, 10_000)
        h.merge_entries(b.to_device())
        o.merge_entries(b)
        rh, ro = h.trace(True), o.trace(True)
        _same(rh, ro)
        if k >= 1:                                     # roots + busy + mail in flight ~ 11 %
            assert 0.09 * ro.n_live < ro.pseudo_roots < 0.13 * ro.n_live
    assert h.export() == o.export()
    assert h.total_actors_seen() == o.total_actors_seen()


def test_c2_shape_busy_wakeups_match_oracle(hip_mod, oracle_mod):
    """C2 at 1/10 scale with the §8d wakeup: 10 % busy / in flight at every cut."""
    actors = 1_000_000
    w = world.World(seed=0x5EED + 2)
    w.bulk_graph(actors, 10 * actors, alpha=2.1, n_roots=actors // 1000, cap=100000)
    h = hip_mod.ShadowGraph(vertex_capacity=actors, edge_capacity=12 * actors)
    o = oracle_mod.OracleGraph()
    for b in w.batches(1 << 20):
        h.merge_entries(b)
        o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    for k in range(3):
        b = busy_wakeup(w, actors, actors // 10)
        h.merge_entries(b.to_device())
        o.merge_entries(b)
        rh, ro = h.trace(True), o.trace(True)
        _same(rh, ro)
        assert rh.edges_scanned == ro.edges_scanned
    assert ro.pseudo_roots > 0.09 * ro.n_live
    assert h.total_actors_seen() == o.total_actors_seen()


@pytest.mark.parametrize("actors,edges,batch,wakeups", [
    (100_000, 1_000_000, 10_000, 6),       # power law at C1 size, quiet wakeups
    (1_000_000, 10_000_000, 100_000, 2),   # C2 shape at 1/10 scale, quiet wakeups
])
def test_power_law_wakeups_match_oracle(hip_mod, oracle_mod, actors, edges, batch, wakeups):
    w = world.World(seed=0x5EED + 1)
    w.bulk_graph(actors, edges, alpha=2.1, n_roots=max(1, actors // 100))
    h = hip_mod.ShadowGraph(vertex_capacity=actors, edge_capacity=edges)
    o = oracle_mod.OracleGraph()
    for b in w.batches(1 << 20):
        h.merge_entries(b)
        o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    for _ in range(wakeups):
        b = w.wakeup_batch(batch)
        h.merge_entries(b.to_device())
        o.merge_entries(b)
        _same(h.trace(True), o.trace(True))
    if actors <= 100_000:
        assert h.export() == o.export()
    assert h.total_actors_seen() == o.total_actors_seen()


@pytest.mark.parametrize("div", ["16", "0"])
def test_slot_reuse_batches_through_grows(hip_mod, oracle_mod, monkeypatch, div):
    """Slot reuse as the library runs it (CRGC_SLOT_REUSE_DIV=16: the swept
    slots wait listed until they are 1/16 of the range, then one purge) on a
    power-law graph loaded in small batches into a graph at its minimum
    capacity, so it grows in place (crgc_api.hip grow) with garbage slots
    still listed, then wakeups that collect and spawn; every trace and the
    final graph equal to the oracle's (ShadowGraph.java:205-289, :276)."""
    monkeypatch.setenv("CRGC_SLOT_REUSE_DIV", div)
    w = world.World(seed=0x5EED + 9)
    w.bulk_graph(40_000, 400_000, alpha=2.1, n_roots=400)
    h = hip_mod.ShadowGraph(vertex_capacity=1000, edge_capacity=10_000)
    o = oracle_mod.OracleGraph()
    for b in w.batches(1 << 13):
        h.merge_entries(b)
        o.merge_entries(b)
        _same(h.trace(True), o.trace(True))
    for _ in range(8):
        b = w.wakeup_batch(4000)
        h.merge_entries(b.to_device())
        o.merge_entries(b)
        _same(h.trace(True), o.trace(True))
    assert h.export() == o.export()
    assert h.total_actors_seen() == o.total_actors_seen()
    u = h.usage()
    assert u["grows"] >= 1, u


@pytest.mark.parametrize("chain_after", ["16", "64", "0", "2"])
def test_c3_deep_chains_and_dead_rings(hip_mod, oracle_mod, monkeypatch, chain_after):
    """Chains walked by k_tail (CRGC_CHAIN_AFTER=0) or handed to chain mode
    (pointer jumping) after 16 (the default) / 64 / 2 links: the same marks."""
    monkeypatch.setenv("CRGC_CHAIN_AFTER", chain_after)
    w = world.World(seed=0x5EED + 3)
    w.chain_graph(n_chains=20, chain_len=3000, n_sup_chains=5, sup_depth=400,
                  n_rings=30, ring_len=60)
    h = hip_mod.ShadowGraph()
    o = oracle_mod.OracleGraph()
    for b in w.batches(50_000):
        h.merge_entries(b)
        o.merge_entries(b)
    rh, ro = h.trace(True), o.trace(True)
    _same(rh, ro)
    assert len(ro.garbage) == 30 * 60 and len(ro.kill) == 30 * 60
    assert rh.levels >= 1
    assert h.export() == o.export()
    _same(h.trace(True), o.trace(True))      # again, nothing to collect
    assert h.count_reachable_from(1) == o.count_reachable_from(1)


def test_c5_cluster_deltas_and_undo(hip_mod, oracle_mod):
    cw = cluster.ClusterWorld(seed=9, n_nodes=8, max_actors=3000)
    h = hip_mod.ShadowGraph()
    o = oracle_mod.OracleGraph()
    merged = []
    for _ in range(8):
        cw.run_turns(500)
        own, deltas = cw.flush(0)
        for k, g in deltas:
            b = g.to_batch()
            h.merge_deltas(b)
            o.merge_deltas(b)
            merged.append((k, g))
        h.merge_entries(own)
        o.merge_entries(own)
        _same(h.trace(True), o.trace(True))
    assert h.export() == o.export()
    # node 8 (index 7) is downed: replay its undo log, then trace
    log = cw.undo_log(7, merged).to_batch(restrict_to=set(o.export().vertices))
    h.merge_undo(log)
    o.merge_undo(log)
    assert h.export() == o.export()
    assert h.count_reachable_from(8) == o.count_reachable_from(8)
    _same(h.trace(True), o.trace(True))


@pytest.mark.slow
def test_c2_full_size_properties(hip_mod):
    """1e7 actors / 1e8 edges: properties that need no oracle."""
    w = world.World(seed=0x5EED + 2)
    w.bulk_graph(10_000_000, 100_000_000, alpha=2.1, n_roots=10_000)
    h = hip_mod.ShadowGraph(vertex_capacity=12_000_000, edge_capacity=120_000_000)
    for b in w.batches(1_000_000):
        h.merge_entries(b.to_device())
    seen = h.total_actors_seen()
    r0 = h.trace(True)
    assert r0.n_live + len(r0.garbage) == seen          # every shadow is live or garbage
    for _ in range(2):
        b = busy_wakeup(w, 10_000_000, 1_000_000)
        h.merge_entries(b.to_device())
        pre = h.live_count()
        r = h.trace(True)
        g = r.garbage
        assert len(np.unique(g)) == len(g)                 # no duplicates
        assert r.kill_set() <= r.garbage_set()             # kills are garbage
        assert r.n_live + len(g) == pre                    # partition of the graph
        assert h.live_count() == r.n_live
    # idempotence: with no new entries a second trace finds no garbage
    r2 = h.trace(True)
    assert len(r2.garbage) == 0 and r2.n_live == h.live_count()
