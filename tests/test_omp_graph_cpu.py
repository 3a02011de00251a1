"""The strong CPU baseline (oracle/omp_graph.cpp) computes what the oracle
computes: per wakeup, the same garbage and kill SETS and the same live /
pseudo-root / traced-edge counts on the C1 stream and a C2-shaped one.  This
pins it, so bench.py's cpu_baseline times the same work as the GPU line and the
full-size GPU parity tests (tests/test_hip_full_size.py) may use it as the
checker where the single-thread oracle would take too long."""
import pytest

import world


def _c1():
    w = world.World(seed=0x5EED + 1)
    w.set_mix(send=0.2, share=0.2, release=0.2, spawn=0.2, actions_per_msg=2.0)
    w.uniform_graph(50_000, mean_acq=8.0, n_roots=500, dead_frac=0.05)
    return w, 50_000


def _c2():
    w = world.World(seed=0x5EED + 2)
    w.bulk_graph(50_000, 500_000, alpha=2.1, n_roots=50, cap=100000)
    return w, 50_000


@pytest.mark.parametrize("make", [_c1, _c2], ids=["c1", "c2"])
def test_omp_graph_matches_oracle(oracle_mod, make):
    w, V = make()
    o, p = oracle_mod.OracleGraph(), oracle_mod.OmpGraph(threads=4)
    for b in w.batches(1 << 16):
        o.merge_entries(b)
        p.merge_entries(b)
    for k in range(5):
        if k:
            b = w.wakeup(V // 10, busy=V * 9 // 100, pending=V // 100)
            o.merge_entries(b)
            p.merge_entries(b)
        ro, rp = o.trace(True), p.trace(True, ids=True)
        assert (len(ro.garbage), len(ro.kill), ro.n_live, ro.pseudo_roots, ro.edges_scanned) == \
            (rp["garbage"], rp["kill"], rp["live"], rp["pseudo_roots"], rp["edges_scanned"]), k
        assert ro.garbage_set() == set(rp["garbage_ids"].tolist()), k
        assert ro.kill_set() == set(rp["kill_ids"].tolist()), k


def _same(ro, rp, what):
    assert (len(ro.garbage), len(ro.kill), ro.n_live, ro.pseudo_roots, ro.edges_scanned) == \
        (rp["garbage"], rp["kill"], rp["live"], rp["pseudo_roots"], rp["edges_scanned"]), what
    assert ro.garbage_set() == set(rp["garbage_ids"].tolist()), what
    assert ro.kill_set() == set(rp["kill_ids"].tolist()), what


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_omp_graph_deltas_and_undo_match_oracle(oracle_mod, seed):
    """The engine's mergeDelta / mergeUndoLog (round 6; ShadowGraph.java:127-174)
    against the oracle on the fuzz streams of the GPU parity tests: entries,
    delta batches every other step, an undo log (halting a node, possibly the
    reference's CME) — the same sets and counts after every step."""
    import fuzz
    from crgc_hip import abi
    o, p = oracle_mod.OracleGraph(), oracle_mod.OmpGraph(threads=4)
    fz = fuzz.Fuzz(seed)
    for step in range(14):
        eb = fz.entries(200 + 50 * step)
        o.merge_entries(eb)
        p.merge_entries(eb)
        if step % 2 == 1:
            db = fz.deltas(5)
            o.merge_deltas(db)
            p.merge_deltas(db)
        if step in (5, 9):
            ub = fz.undo(o.export().vertices.keys())
            codes = []
            for g in (o, p):
                try:
                    g.merge_undo(ub)
                    codes.append(0)
                except abi.CrgcError as e:
                    codes.append(e.code)
            assert codes[0] == codes[1], (step, codes)
        _same(o.trace(True), p.trace(True, ids=True), step)
        fz.sync(o.export())


def test_omp_graph_c5_cluster_stream_matches_oracle(oracle_mod):
    """C5's shape at a small size: node 1's own entries plus the other nodes'
    DeltaGraphs (workload/world.py deltas_of), then node 8 downed — its last
    deltas undone (workload/delta.py undo_of)."""
    from crgc_hip import DeltaBatch, abi
    nodes, V, E, B = 8, 4000, 40_000, 400
    ws = [world.World(seed=0x5EED + 5 + 1000 * k, location=k + 1) for k in range(nodes)]
    for w in ws:
        w.bulk_graph(V, E, alpha=2.1, n_roots=max(1, V // 1000), cap=100000)
    o, p = oracle_mod.OracleGraph(), oracle_mod.OmpGraph(threads=4)
    for k, w in enumerate(ws):
        for b in w.batches(1 << 16):
            if k == 0:
                o.merge_entries(b)
                p.merge_entries(b)
            else:
                d = world.deltas_of(b)[0]
                o.merge_deltas(d)
                p.merge_deltas(d)
    _same(o.trace(True), p.trace(True, ids=True), "load")
    parts = None
    for step in range(3):
        own = ws[0].wakeup_batch(B)
        parts = [world.deltas_of(ws[k].wakeup_batch(B))[0] for k in range(1, nodes)]
        d = DeltaBatch.concat(parts)
        for g in (o, p):
            g.merge_deltas(d)
            g.merge_entries(own)
        _same(o.trace(True), p.trace(True, ids=True), step)
    log = world.undo_of(parts[-1], nodes)
    codes = []
    for g in (o, p):
        try:
            g.merge_undo(log)
            codes.append(0)
        except abi.CrgcError as e:
            codes.append(e.code)
    assert codes[0] == codes[1]
    _same(o.trace(True), p.trace(True, ids=True), "downed node")
