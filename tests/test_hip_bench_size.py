"""Parity at the bench's own sizes where the oracle can afford it.

* C3 exactly as `bench.py --workload c3` builds it (100 chains x 1e4 links, 10
  supervisor chains of depth 1e3, 100 dead rings of 100, seed 0x5EED+3): the
  oracle traces it in ~60 ms.
* C5 as `bench.py --workload c5` builds it, at 1/10 scale (8 nodes x 125 000
  actors, 12 500-entry batches per node and wakeup): node 1 merges its own
  entries and the other seven nodes' DeltaGraphs, folds them into the senders'
  UndoLogs on the device, traces; then node 8 is downed and its last deltas are
  undone (crgc_merge_undo_acc = ShadowGraph.mergeUndoLog) before a trace.
* Sharded C3 at G = 8 logical shards with 3 000-link chains.

Every trace is compared with the oracle (ShadowGraph.java:205-289) on garbage /
kill sets, counts, pseudo-roots and scanned edges; merges on the exported state
(ShadowGraph.java:64-174) where the export fits in host memory quickly.
"""
import pytest

import world
from test_hip_undo_acc import _canon

pytestmark = pytest.mark.gpu


def _same(rh, ro):
    assert rh.garbage_set() == ro.garbage_set()
    assert rh.kill_set() == ro.kill_set()
    assert len(rh.garbage) == len(ro.garbage) and len(rh.kill) == len(ro.kill)
    assert rh.n_live == ro.n_live
    assert rh.pseudo_roots == ro.pseudo_roots
    assert rh.sup_edges == ro.sup_edges
    assert rh.edges_scanned == ro.edges_scanned


def test_c3_bench_graph_full_size(hip_mod, oracle_mod):
    w = world.World(seed=0x5EED + 3)
    w.chain_graph(n_chains=100, chain_len=10000, n_sup_chains=10, sup_depth=1000,
                  n_rings=100, ring_len=100)
    h, o = hip_mod.ShadowGraph(), oracle_mod.OracleGraph()
    for b in w.batches(1 << 20):
        h.merge_entries(b.to_device())
        o.merge_entries(b)
    assert h.export() == o.export()
    rh, ro = h.trace(True), o.trace(True)
    _same(rh, ro)
    assert len(ro.garbage) == 100 * 100           # the dead rings
    assert ro.n_live > 100 * 10000                # every chain link is live
    for _ in range(2):                            # the bench's timed traces: nothing more to collect
        rh, ro = h.trace(True), o.trace(True)
        _same(rh, ro)
        assert len(ro.garbage) == 0
    assert h.count_reachable_from(1) == o.count_reachable_from(1)
    assert h.total_actors_seen() == o.total_actors_seen()


def _add_undo(want, u):
    for a, (m, refs) in _canon(u).items():
        pm, pr = want.get(a, (0, {}))
        for t, c in refs.items():
            pr[t] = pr.get(t, 0) + c
            if pr[t] == 0:
                del pr[t]
        want[a] = (pm + m, pr)


def test_c5_bench_construction_tenth_scale(hip_mod, oracle_mod):
    from crgc_hip import DeltaBatch, abi
    nodes, V, E, B = 8, 125_000, 1_250_000, 12_500
    ws = [world.World(seed=0x5EED + 5 + 1000 * k, location=k + 1) for k in range(nodes)]
    for w in ws:
        w.bulk_graph(V, E, alpha=2.1, n_roots=max(1, V // 1000), cap=100000)
    h = hip_mod.ShadowGraph(vertex_capacity=int(nodes * V * 1.2), edge_capacity=int(nodes * E * 1.2))
    o = oracle_mod.OracleGraph()
    accs = [h.undo_accumulator(k + 1) for k in range(1, nodes)]
    want = [dict() for _ in range(1, nodes)]
    for k, w in enumerate(ws):
        for b in w.batches(1 << 20):
            if k == 0:
                h.merge_entries(b.to_device())
                o.merge_entries(b)
            else:
                d = world.deltas_of(b)[0]
                dd = d.to_device()
                h.merge_deltas(dd)
                o.merge_deltas(d)
                accs[k - 1].fold_deltas(dd)
                _add_undo(want[k - 1], world.undo_of(d, k + 1))
    _same(h.trace(True), o.trace(True))

    def wakeup():
        own = ws[0].wakeup_batch(B)
        parts = [world.deltas_of(ws[k].wakeup_batch(B))[0] for k in range(1, nodes)]
        deltas = DeltaBatch.concat(parts)
        h.merge_deltas(deltas.to_device())
        h.merge_entries(own.to_device())
        o.merge_deltas(deltas)
        o.merge_entries(own)
        return parts

    for _ in range(3):
        parts = wakeup()
        for k, (acc, p) in enumerate(zip(accs, parts)):
            acc.fold_deltas(p.to_device())
            _add_undo(want[k], world.undo_of(p, k + 2))
        rh, ro = h.trace(True), o.trace(True)
        _same(rh, ro)
        assert ro.pseudo_roots > 0 and ro.edges_scanned > 0
    for acc, wnt in zip(accs, want):
        assert _canon(acc.export()) == wnt
    assert h.total_actors_seen() == o.total_actors_seen()
    # node 8 is downed: its deltas merged since the last trace are undone, then trace
    parts = wakeup()
    last8 = h.undo_accumulator(nodes)
    last8.fold_deltas(parts[-1].to_device())
    log = world.undo_of(parts[-1], nodes)
    assert _canon(last8.export()) == _canon(log)
    try:
        o.merge_undo(log)
        cme = None
    except abi.CrgcError as e:
        cme = e.code
    if cme is None:
        h.merge_undo_acc(last8)
        assert h.count_reachable_from(nodes) == o.count_reachable_from(nodes)
        _same(h.trace(True), o.trace(True))
    else:
        with pytest.raises(abi.CrgcError) as e:
            h.merge_undo_acc(last8)
        assert e.value.code == cme


def test_c3_chains_eight_shards(hip_mod, oracle_mod):
    g = hip_mod.ShardedShadowGraph(8)
    try:
        w = world.World(seed=0x5EED + 3)
        w.chain_graph(n_chains=6, chain_len=3000, n_sup_chains=3, sup_depth=500,
                      n_rings=10, ring_len=60)
        o = oracle_mod.OracleGraph()
        for b in w.batches(1 << 16):
            g.merge_entries(b, split=True)
            o.merge_entries(b)
        assert g.export() == o.export()
        rh, ro = g.trace(True), o.trace(True)
        _same(rh, ro)
        assert len(ro.garbage) == 10 * 60
        # deep marks finish in the replicated chain closure (crgc_xchain.hip):
        # rounds grow with log2 of the depth, not with the cross-shard links
        assert rh.rounds <= 2 * 12 + 4, rh.rounds
        rh2, ro2 = g.trace(True), o.trace(True)
        _same(rh2, ro2)
        assert rh2.rounds <= 2 * 12 + 4, rh2.rounds
        assert g.export() == o.export()
    finally:
        g.close()


@pytest.mark.parametrize("reg_chunks,sdma", [("1", "0"), ("2", "0"), ("1", "1"), ("2", "1")])
def test_large_host_batches_chunked_and_registered(hip_mod, oracle_mod, monkeypatch, reg_chunks, sdma):
    """Host batches of >= 2^19 entries take the merge's host paths (crgc_api.hip
    crgc_merge_entries): a pageable batch is copied and merged in chunks, one
    merge per chunk with its own epoch (merge_entries_chunked); a batch in a
    buffer registered with crgc_host_register is read over PCIe by
    k_copy_ranges, in one piece (the default) or in CRGC_CHUNK_REG = 2 chunks.  Both graphs must
    equal the oracle's after every merge, and their traces too
    (ShadowGraph.java:64-156, 205-289)."""
    from crgc_hip import HostArena
    monkeypatch.setenv("CRGC_BIN_MIN_SLOTS", "0")  # and the pseudo-root level binned at this size
    monkeypatch.setenv("CRGC_CHUNK_REG", reg_chunks)
    monkeypatch.setenv("CRGC_REG_SDMA", sdma)  # 1: the chunks by DMA (one span each) instead of k_copy_ranges
    w = world.World(seed=0x5EED + 7)
    w.bulk_graph(200_000, 2_000_000)
    hp, hr, o = hip_mod.ShadowGraph(), hip_mod.ShadowGraph(), oracle_mod.OracleGraph()
    loads = list(w.batches(1 << 20))
    for b in loads:
        hp.merge_entries(b.to_device())
        hr.merge_entries(b.to_device())
        o.merge_entries(b)
    big = [w.wakeup(600_000, busy=18_000, pending=2_000) for _ in range(2)]
    assert all(len(b.self) >= 1 << 19 for b in big)
    arena = HostArena(max(b.nbytes() for b in big) * 1.1 + (1 << 20))
    hr.register_host(arena.buf)
    for b in big:
        hp.merge_entries(b)                # pageable: chunked
        hr.merge_entries(arena.pack(b))    # registered: kernel copies
        o.merge_entries(b)
        want = o.export()
        assert hp.export() == want
        assert hr.export() == want
        ro = o.trace(True)
        _same(hp.trace(True), ro)
        _same(hr.trace(True), ro)
    hr.unregister_host(arena.buf)


@pytest.mark.parametrize("sdma", ["0", "1"])
def test_drain_loop_chunks_merged_async_from_registered_arena(hip_mod, oracle_mod, monkeypatch, sdma):
    """crgc_merge_entries_async: the drain loop packs a wakeup's entries into a
    registered arena chunk by chunk (LocalGC.scala:152-172) and hands each chunk
    over as soon as it is packed; the merges run while the next chunk is packed,
    and the arena is reused only after the trace.  Chunks merge in call order,
    so the graph equals the oracle's after the whole batch, and the traces too."""
    from crgc_hip import HostArena
    monkeypatch.setenv("CRGC_REG_SDMA", sdma)
    w = world.World(seed=0x5EED + 9)
    w.bulk_graph(100_000, 1_000_000)
    h, o = hip_mod.ShadowGraph(), oracle_mod.OracleGraph()
    for b in w.batches(1 << 20):
        h.merge_entries(b.to_device())
        o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    wake = [w.wakeup(100_000, busy=9_000, pending=1_000) for _ in range(3)]
    arena = HostArena(max(b.nbytes() for b in wake) * 1.2 + (1 << 22))
    h.register_host(arena.buf)
    try:
        for b in wake:
            at = 0
            n = len(b.self)
            for lo in range(0, n, 30_000):          # 4 chunks, the last short
                hb = arena.pack(b.slice(lo, min(n, lo + 30_000)), at)
                at = (arena.end + 255) & ~255
                h.merge_entries_async(hb)
            o.merge_entries(b)
            ro = o.trace(True)
            _same(h.trace(True), ro)
            assert h.export() == o.export()
    finally:
        h.unregister_host(arena.buf)
