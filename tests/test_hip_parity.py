"""Parity of the HIP shadow graph against the CPU oracle (bit-exact sets/state).

Every test drives the product through its C ABI (crgc_hip.ShadowGraph ->
libcrgc_hip.so) and checks it against oracle.OracleGraph on the same stream.
"""
import numpy as np
import pytest

import fuzz
import kats
from crgc_hip import abi

pytestmark = pytest.mark.gpu


def _pair(hip_mod, oracle_mod, **kw):
    return hip_mod.ShadowGraph(**kw), oracle_mod.OracleGraph()


def _same_trace(rh, ro):
    assert rh.garbage_set() == ro.garbage_set()
    assert rh.kill_set() == ro.kill_set()
    assert len(rh.garbage) == len(ro.garbage), "duplicate garbage ids"
    assert len(rh.kill) == len(ro.kill), "duplicate kill ids"
    assert rh.n_live == ro.n_live
    assert rh.pseudo_roots == ro.pseudo_roots
    assert rh.sup_edges == ro.sup_edges
    assert rh.edges_scanned == ro.edges_scanned


# Traversal directions.  "pull" forces every level after the roots to pull
# (in-candidate scan) and "push" disables pulling; "auto" is the product
# default (pull only for large dense levels, i.e. push at these sizes, and
# k_tail once a sparse level's frontier is narrow).
DIRECTIONS = {
    "auto": {},
    "push": {"CRGC_PULL": "0", "CRGC_SPARSE_THRESH": "0"},
    "pull": {"CRGC_PULL": "1", "CRGC_PULL_THRESH": "1", "CRGC_SPARSE_THRESH": "0"},
    # narrow-frontier workgroup (k_tail) off, and on at every sparse level with
    # a bail back to the level kernels whenever a round finds more than 3
    "notail": {"CRGC_TAIL": "0"},
    "tailbail": {"CRGC_TAIL_START": "65536", "CRGC_TAIL_MAX": "3"},
    # k_tail at every sparse level, handing to chain mode (pointer jumping,
    # crgc_chain.hip) after a one-link walk
    "chains": {"CRGC_TAIL_START": "65536", "CRGC_CHAIN_AFTER": "1"},
}


@pytest.fixture(params=sorted(DIRECTIONS))
def direction(request, monkeypatch):
    for k, v in DIRECTIONS[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


@pytest.mark.parametrize("name", sorted(kats.SCENARIOS))
def test_kat_scenarios_on_hip(hip_mod, name):
    g = hip_mod.ShadowGraph()
    kats.run_scenario(g, kats.SCENARIOS[name]())


@pytest.mark.parametrize("seed", [1, 2])
def test_random_spec_on_hip(hip_mod, oracle_mod, seed):
    g = hip_mod.ShadowGraph()
    collected, everyone = kats.run_random(g, seed=seed, max_actors=400)
    assert collected == everyone


def test_random_spec_hip_matches_oracle_every_wakeup(hip_mod, oracle_mod, direction):
    w = kats.RandomWorld(seed=7, max_actors=600, wake_every=13)
    h, o = _pair(hip_mod, oracle_mod)
    for batch in w.steps():
        h.merge_entries(batch)
        o.merge_entries(batch)
        assert h.export() == o.export()
        rh, ro = h.trace(True), o.trace(True)
        _same_trace(rh, ro)
        w.kill(ro.kill_set())
    assert h.total_actors_seen() == o.total_actors_seen()


@pytest.mark.parametrize("seed,cap", [(11, 0), (12, 0), (13, 64)])
def test_fuzz_entries_deltas_undo(hip_mod, oracle_mod, seed, cap, direction):
    # cap=64 starts from a tiny graph so rebuilds (compaction) happen often
    h, o = _pair(hip_mod, oracle_mod, vertex_capacity=cap, edge_capacity=cap)
    fz = fuzz.Fuzz(seed)
    for step in range(14):
        eb = fz.entries(200 + 50 * step)
        h.merge_entries(eb); o.merge_entries(eb)
        if step % 2 == 1:
            db = fz.deltas(5)
            h.merge_deltas(db); o.merge_deltas(db)
        if step == 9:
            ub = fz.undo(o.export().vertices.keys())
            h.merge_undo(ub); o.merge_undo(ub)
        st = o.export()
        assert h.export() == st
        for loc in (1, 2, 3):
            assert h.count_reachable_from(loc) == o.count_reachable_from(loc)
        assert sorted(h.startWave().tolist()) == sorted(o.local_roots().tolist())
        rh, ro = h.trace(True), o.trace(True)
        _same_trace(rh, ro)
        fz.sync(o.export())
    assert h.total_actors_seen() == o.total_actors_seen()
    assert h.export() == o.export()


def test_should_kill_false_reports_garbage_but_no_kills(hip_mod, oracle_mod):
    h, o = _pair(hip_mod, oracle_mod)
    for st in kats.simple_actor():
        if st[0] == "merge":
            h.merge_entries(st[1]); o.merge_entries(st[1])
        else:
            rh, ro = h.trace(False), o.trace(False)
            _same_trace(rh, ro)
            assert len(rh.kill) == 0


def test_null_supervisor_is_reported_like_the_reference_npe(hip_mod, oracle_mod):
    from crgc_hip import Entry, EntryBatch
    # A local, non-root actor that was never spawned and is not referenced.
    a = (1 << 48) | 77
    b = EntryBatch.from_entries([Entry(self=a)])
    h, o = _pair(hip_mod, oracle_mod)
    h.merge_entries(b); o.merge_entries(b)
    with pytest.raises(abi.CrgcError) as eo:
        o.trace(True)
    assert eo.value.code == abi.E_NULL_SUPERVISOR
    with pytest.raises(abi.CrgcError) as eh:
        h.trace(True)
    assert eh.value.code == abi.E_NULL_SUPERVISOR


def test_undo_naming_unknown_actor_is_reported_like_the_reference_cme(hip_mod, oracle_mod):
    from crgc_hip import Entry, EntryBatch, UndoBatch
    r = (1 << 48) | 1
    b = EntryBatch.from_entries([Entry(self=r, isRoot=True, createdOwners=[r], createdTargets=[r])])
    h, o = _pair(hip_mod, oracle_mod)
    h.merge_entries(b); o.merge_entries(b)
    log = UndoBatch.from_fields(3, [(r, 1, [((3 << 48) | 9, 1)])])
    for g in (h, o):
        with pytest.raises(abi.CrgcError) as e:
            g.merge_undo(log)
        assert e.value.code == abi.E_UNDO_NEW_SHADOW
    assert h.export() == o.export()  # nothing was applied


def test_reserved_ids_are_rejected(hip_mod):
    from crgc_hip import Entry, EntryBatch
    g = hip_mod.ShadowGraph()
    g.merge_entries(EntryBatch.from_entries([Entry(self=abi.NO_ACTOR)]))
    with pytest.raises(abi.CrgcError) as e:
        g.trace(True)
    assert e.value.code == abi.E_INVAL


def test_device_resident_batches(hip_mod, oracle_mod):
    w = kats.RandomWorld(seed=3, max_actors=300, wake_every=17)
    h, o = _pair(hip_mod, oracle_mod)
    for batch in w.steps():
        h.merge_entries(batch.to_device())
        o.merge_entries(batch)
        _same_trace(h.trace(True), o.trace(True))


def test_empty_graph_and_empty_batches(hip_mod, oracle_mod):
    from crgc_hip import EntryBatch, DeltaBatch
    h, o = _pair(hip_mod, oracle_mod)
    h.merge_entries(EntryBatch.empty()); o.merge_entries(EntryBatch.empty())
    h.merge_deltas(DeltaBatch.from_rows([])); o.merge_deltas(DeltaBatch.from_rows([]))
    _same_trace(h.trace(True), o.trace(True))
    assert h.live_count() == 0


def test_last_trace_survives_the_compaction_after_a_trace(hip_mod, oracle_mod):
    """Two-phase trace: crgc_trace with no buffers, then
    crgc_last_trace.  A trace that leaves dead slots outnumbering live ones
    compacts the graph before it returns; the retained lists must survive it."""
    import world
    w = world.World(seed=0x5EED + 21)
    # 1 live chain, 800 dead rings of 100: slot_top > 65536 and dead >> live
    w.chain_graph(n_chains=1, chain_len=1000, n_sup_chains=0, sup_depth=0,
                  n_rings=800, ring_len=100)
    h, o = _pair(hip_mod, oracle_mod)
    for b in w.batches(1 << 20):
        h.merge_entries(b)
        o.merge_entries(b)
    r, ng, nk = h.trace_counts(True)          # no id buffers: counts only
    ro = o.trace(True)
    assert ng == len(ro.garbage) == 80_000 and nk == len(ro.kill)
    assert h.live_count() == ro.n_live         # the compaction ran
    g, k = h.last_trace()
    assert set(g.tolist()) == ro.garbage_set() and len(g) == ng
    assert set(k.tolist()) == ro.kill_set() and len(k) == nk
    # and once more after a merge that grows the graph past its capacity
    w.chain_graph(n_chains=1, chain_len=200_000, n_sup_chains=0, sup_depth=0, n_rings=0, ring_len=0)
    for b in w.batches(1 << 20):
        h.merge_entries(b)
        o.merge_entries(b)
    g2, k2 = h.last_trace()
    assert set(g2.tolist()) == ro.garbage_set() and set(k2.tolist()) == ro.kill_set()
    _same_trace(h.trace(True), o.trace(True))


@pytest.mark.parametrize("buckets_log2", ["1", "3"])
def test_edge_buckets_in_several_rounds(hip_mod, oracle_mod, buckets_log2, monkeypatch):
    """Two or eight owner / target buckets: every bucket workgroup takes its
    atoms in several 1024-atom rounds, so pairs repeat across rounds, edges
    inserted in one round are updated (and flip sign) in the next, and segments
    grow more than once per merge — still bit-exact, state included."""
    monkeypatch.setenv("CRGC_BUCKETS_LOG2", buckets_log2)
    h, o = _pair(hip_mod, oracle_mod)
    fz = fuzz.Fuzz(17)
    for step in range(8):
        eb = fz.entries(2000 + 500 * step)
        h.merge_entries(eb); o.merge_entries(eb)
        db = fz.deltas(40)
        h.merge_deltas(db); o.merge_deltas(db)
        assert h.export() == o.export()
        _same_trace(h.trace(True), o.trace(True))
        fz.sync(o.export())
    assert h.export() == o.export()


def test_registered_host_arena_matches_oracle(hip_mod, oracle_mod):
    """Host batches packed into a buffer pinned by crgc_host_register (the JNI
    shim's reused direct buffers) merge exactly like any host batch; an
    overlapping registration is refused."""
    from crgc_hip import HostArena
    h, o = _pair(hip_mod, oracle_mod)
    arena = HostArena(8 << 20)
    h.register_host(arena.buf)
    with pytest.raises(abi.CrgcError) as e:
        h.register_host(arena.buf[4096:8192])
    assert e.value.code == abi.E_INVAL
    fz = fuzz.Fuzz(23)
    for step in range(6):
        eb = fz.entries(3000)
        h.merge_entries(arena.pack(eb))
        o.merge_entries(eb)
        assert h.export() == o.export()
        _same_trace(h.trace(True), o.trace(True))
        fz.sync(o.export())
    h.unregister_host(arena.buf)
    with pytest.raises(abi.CrgcError):
        h.unregister_host(arena.buf)


@pytest.mark.parametrize("pull", ["0", "1000000"])
def test_fan_in_candidate_overflow(hip_mod, oracle_mod, monkeypatch, pull):
    """Thousands of new in-edges to a few targets in one merge: their reverse
    candidate segments overflow (k_rv_grow / k_rv_place), some of those edges
    change sign again within the same merge's later rounds (CRGC_BUCKETS_LOG2=1:
    two owner buckets, many rounds), and every level pulls (CRGC_ALPHA) so the
    marks depend on the candidates."""
    from crgc_hip import Entry, EntryBatch
    monkeypatch.setenv("CRGC_ALPHA", pull)
    monkeypatch.setenv("CRGC_BUCKETS_LOG2", "1")
    h, o = _pair(hip_mod, oracle_mod)
    loc = 1 << 48
    root = loc | 1
    hubs = [loc | (2 + k) for k in range(3)]
    owners = [loc | (100 + k) for k in range(3000)]
    first = [Entry(self=root, isRoot=True, spawnedActors=hubs,
                   createdOwners=[root] * 2, createdTargets=hubs[:2])]
    # the root spawns every owner (F records per entry) and keeps refs to them
    for k in range(0, len(owners), 4):
        first.append(Entry(self=root, isRoot=True, spawnedActors=owners[k:k + 4],
                           createdOwners=[root] * len(owners[k:k + 4]), createdTargets=owners[k:k + 4]))
    b0 = EntryBatch.from_entries(first)
    h.merge_entries(b0); o.merge_entries(b0)
    for wake in range(4):
        es = []
        for i, ow in enumerate(owners):
            if wake == 0 or (wake == 3 and i % 2):  # refs to every hub: new keys, then 0 -> 1
                es.append(Entry(self=root, isRoot=True, createdOwners=[ow] * 3, createdTargets=hubs))
            if wake in (1, 2) and i % 2:  # released again: 1 -> 0 on one hub per wakeup
                es.append(Entry(self=ow, updatedRefs=[hubs[wake]], updatedInfos=[1]))
        b = EntryBatch.from_entries(es)
        h.merge_entries(b); o.merge_entries(b)
        assert h.export() == o.export()
        _same_trace(h.trace(True), o.trace(True))


def test_entry_field_size_above_255(hip_mod, oracle_mod):
    """uigc.crgc.entry-field-size is any int in the reference (Context.java:14):
    F = 300, and 512 root entries that all spawn the same 300 children — about
    76 500 last-write-wins supervisor conflicts in the first 256-entry block,
    more than round 3's 16-bit per-block count could hold.  Every
    child's supervisor must be the last spawner in batch order (:101-102)."""
    from crgc_hip import Entry, EntryBatch
    F = 300
    h = hip_mod.ShadowGraph(entry_field_size=F)
    o = oracle_mod.OracleGraph(entry_field_size=F)
    loc = 1 << 48
    root = loc | 1
    parents = [loc | (10 + i) for i in range(512)]
    kids = [loc | (10_000 + j) for j in range(F)]
    es = [Entry(self=root, isRoot=True, spawnedActors=parents[:F]),      # supervisor of the parents
          Entry(self=root, isRoot=True, spawnedActors=parents[F:])]
    es += [Entry(self=p, isRoot=True, spawnedActors=kids, createdOwners=[p], createdTargets=[kids[i % F]])
           for i, p in enumerate(parents)]
    b = EntryBatch.from_entries(es)
    h.merge_entries(b)
    o.merge_entries(b)
    st = h.export()
    assert st == o.export()
    assert {st.vertices[k][2] for k in kids} == {parents[-1]}  # (recv, flags, supervisor)
    _same_trace(h.trace(True), o.trace(True))
    # the parents stop being roots and release their refs: only the last one stays
    # live (the kids' supervisor); the others are garbage, killed (their supervisor is live)
    es = [Entry(self=p, updatedRefs=[kids[i % F]], updatedInfos=[1]) for i, p in enumerate(parents)]
    b = EntryBatch.from_entries(es)
    h.merge_entries(b)
    o.merge_entries(b)
    assert h.export() == o.export()
    rh, ro = h.trace(True), o.trace(True)
    _same_trace(rh, ro)
    assert rh.kill_set() == set(parents[:-1])


def test_trace_ids_into_partly_registered_buffer(hip_mod, oracle_mod):
    """the device stores trace ids straight into a caller buffer only
    when the whole capacity lies in one pinned range.  A garbage buffer that
    starts inside a crgc_host_register range and runs past its end gets the ids
    by a stream copy (direct_lists = 0) — a device store there would fault — and
    buffers wholly inside the range get them from the device (direct_lists = 1)."""
    h, o = _pair(hip_mod, oracle_mod)
    arena = np.zeros(1 << 20, np.uint64)        # 8 MiB; the first half is registered
    half = 1 << 19
    h.register_host(arena[:half])
    fz = fuzz.Fuzz(29)
    try:
        for step in range(6):
            eb = fz.entries(3000)
            h.merge_entries(eb)
            o.merge_entries(eb)
            if step % 2 == 0:
                g, want_direct = arena[half - 64:half + 8192], 0   # runs past the pinned half
            else:
                g, want_direct = arena[8192:8192 + 16384], 1      # wholly pinned
            k = arena[:8192]
            rc, out = h._trace_into(True, g, k)
            assert rc == abi.OK
            ro = o.trace(True)
            assert set(g[:out.n_garbage].tolist()) == ro.garbage_set()
            assert set(k[:out.n_kill].tolist()) == ro.kill_set()
            assert out.n_live == ro.n_live
            assert out.stats.direct_lists == want_direct, step
            assert out.stats.time_query_failures == 0
            fz.sync(o.export())
    finally:
        h.unregister_host(arena[:half])


@pytest.mark.parametrize("seed,cap", [(17, 0), (18, 64)])
def test_device_sub_merges_and_pool_repacks(hip_mod, oracle_mod, monkeypatch, seed, cap):
    """Large device batches merge in sub-merges with rebased offsets (here every
    300 entries: CRGC_DEV_CHUNK), and the pools are repacked before every merge
    (CRGC_REPACK_EACH_MERGE: segments move, slots and tables stay) — alongside
    deltas, undo logs and, at cap 64, rebuilds.  Bit-exact with the oracle."""
    monkeypatch.setenv("CRGC_DEV_CHUNK", "300")
    monkeypatch.setenv("CRGC_REPACK_EACH_MERGE", "1")
    h, o = _pair(hip_mod, oracle_mod, vertex_capacity=cap, edge_capacity=cap)
    fz = fuzz.Fuzz(seed)
    for step in range(10):
        eb = fz.entries(700 + 90 * step)
        h.merge_entries(eb.to_device())
        o.merge_entries(eb)
        if step % 3 == 1:
            db = fz.deltas(5)
            h.merge_deltas(db); o.merge_deltas(db)
        if step == 6:
            ub = fz.undo(o.export().vertices.keys())
            h.merge_undo(ub); o.merge_undo(ub)
        assert h.export() == o.export()
        rh, ro = h.trace(True), o.trace(True)
        _same_trace(rh, ro)
        fz.sync(o.export())
    assert h.total_actors_seen() == o.total_actors_seen()


def test_device_sub_merge_bad_later_boundary_refused_whole(hip_mod, oracle_mod, monkeypatch):
    """a large device batch whose created offsets run backwards at a
    later sub-merge boundary is refused whole (CRGC_E_INVAL) before any
    sub-merge runs — the graph is unchanged and stays usable, as for a host
    batch — instead of being refused after the earlier chunks merged."""
    from crgc_hip.batch import EntryBatch
    monkeypatch.setenv("CRGC_DEV_CHUNK", "300")
    h, o = _pair(hip_mod, oracle_mod)
    fz = fuzz.Fuzz(41)
    eb = fz.entries(2000)
    h.merge_entries(eb.to_device())
    o.merge_entries(eb)
    fz.sync(o.export())
    before = h.export()
    assert before == o.export()
    bad = fz.entries(700)
    co = bad.created_off.copy()
    co[600] = co[700] + 1        # chunk [600, 700) runs backwards; chunk [300, 600) stays legal
    assert co[600] - co[300] <= 300 * 4
    nb = EntryBatch(bad.self, bad.recv_count, bad.flags, co, bad.created_owner, bad.created_target,
                    bad.spawned_off, bad.spawned, bad.updated_off, bad.updated_ref, bad.updated_info)
    with pytest.raises(abi.CrgcError) as ei:
        h.merge_entries(nb.to_device())
    assert ei.value.code == abi.E_INVAL
    assert h.export() == before   # nothing merged, not poisoned
    h.merge_entries(bad.to_device())   # the same entries with their offsets intact
    o.merge_entries(bad)
    assert h.export() == o.export()
    _same_trace(h.trace(True), o.trace(True))


def test_failure_detail_names_the_call(hip_mod):
    """A status code says what failed, crgc_last_error_detail() where: a graph
    whose slot capacity cannot be allocated fails with CRGC_E_NOMEM, and the
    exception carries the call site and the HIP status (crgc_api.hip map_hip_at);
    the next successful call clears it."""
    from crgc_hip import abi
    with pytest.raises(abi.CrgcError) as ei:
        hip_mod.ShadowGraph(vertex_capacity=1 << 40, edge_capacity=1 << 20)
    assert ei.value.code == abi.E_NOMEM
    assert "crgc_api.hip:" in ei.value.detail and "hipErrorOutOfMemory" in ei.value.detail
    g = hip_mod.ShadowGraph(vertex_capacity=1024, edge_capacity=4096)
    g.trace(True)
    assert abi.last_error_detail() == ""


@pytest.mark.parametrize("reuse,div", [("1", "0"), ("1", "16"), ("0", "0")])
def test_swept_slots_reused_match_oracle(hip_mod, oracle_mod, monkeypatch, reuse, div):
    """Slot reuse (crgc_reuse.hip, round 6): after every committed sweep the
    garbage slots are purged of their edges (keys tombstoned, in-edges left
    with count 0, candidates and pull hints made inert), reset, and taken by
    the next merges' new shadows — the reference's shadowMap.remove
    (ShadowGraph.java:276) for dense slots.  A RandomSpec stream collects
    thousands of actors while spawning new ones, so most slots are reused, some
    several times; the graph and every trace must equal the oracle's, and the
    slot range must stay near the live set.  CRGC_SLOT_REUSE=0 is the control
    (slots reclaimed by rebuilds only).  div = 0 purges after every sweep (the
    suite's default, tests/conftest.py); 16 (the library default) lists the
    garbage slots and purges them in batches of 1/16 of the slot range
    (tests/test_hip_configs.py also grows a graph with slots listed)."""
    monkeypatch.setenv("CRGC_SLOT_REUSE", reuse)
    monkeypatch.setenv("CRGC_SLOT_REUSE_DIV", div)
    w = kats.RandomWorld(seed=31, max_actors=3000, wake_every=40)
    h, o = _pair(hip_mod, oracle_mod, vertex_capacity=1 << 16, edge_capacity=1 << 16)
    peak_live, collected = 0, 0
    for batch in w.steps():
        h.merge_entries(batch)
        o.merge_entries(batch)
        assert h.export() == o.export()
        rh, ro = h.trace(True), o.trace(True)
        _same_trace(rh, ro)
        w.kill(ro.kill_set())
        peak_live = max(peak_live, ro.n_live)
        collected += len(ro.garbage)
    assert h.total_actors_seen() == o.total_actors_seen()
    u = h.usage()
    seen = h.total_actors_seen()
    assert collected > seen // 2  # most actors were collected along the way
    if reuse == "1":
        # new shadows took collected shadows' slots: the range stays near the
        # peak live set (plus one wakeup's new shadows), far below the actors seen
        assert u["slot_top"] <= 2 * peak_live + 256 < seen, (u, peak_live, seen)
    else:
        assert u["free_slots"] == 0 and u["slot_top"] == seen, (u, seen)  # (no rebuild below 65536 slots)
    assert u["rebuilds"] == 0, u


def test_swept_slots_reused_with_halted_supervisors(hip_mod, oracle_mod):
    """Halted live shadows are never expanded (ShadowGraph.java:226-229), so a
    sweep can collect their supervisors; before those slots are reused the
    halted shadows' supervisor pointers become SLOT_DEAD (k_sup_fix), and the
    exported supervisor stays the dead actor.  Entries, deltas and an undo log
    (which halts a node's actors) over many wakeups, compared with the oracle
    after every step."""
    h, o = _pair(hip_mod, oracle_mod, vertex_capacity=4096, edge_capacity=4096)
    fz = fuzz.Fuzz(57)
    for step in range(24):
        eb = fz.entries(300)
        h.merge_entries(eb); o.merge_entries(eb)
        if step % 3 == 1:
            db = fz.deltas(6)
            h.merge_deltas(db); o.merge_deltas(db)
        if step in (6, 15):
            ub = fz.undo(o.export().vertices.keys())
            h.merge_undo(ub); o.merge_undo(ub)
        assert h.export() == o.export()
        _same_trace(h.trace(True), o.trace(True))
        fz.sync(o.export())
    assert h.total_actors_seen() == o.total_actors_seen()
    assert h.export() == o.export()
