"""Hash-partitioned shadow graph against the unsharded CPU oracle.

G logical shards run on the one GPU of the test box, each shard a crgc_graph
handle driven by its own host thread, exchanging through the in-process
transport (device copies) — the same protocol the RCCL transport runs with one
process per GPU.  Every check is bit-exact against oracle.OracleGraph (an
unsharded restatement of ShadowGraph.java): the union of the shards' garbage
and kill sets, the sums of their counts, and the union of their exported
state must equal the oracle's, wakeup by wakeup.
"""
import numpy as np
import pytest

import cluster
import fuzz
import kats
import world
from crgc_hip import abi

pytestmark = pytest.mark.gpu


def _same(rh, ro):
    assert rh.garbage_set() == ro.garbage_set()
    assert rh.kill_set() == ro.kill_set()
    assert len(rh.garbage) == len(ro.garbage), "a garbage id reported twice"
    assert len(rh.kill) == len(ro.kill), "a kill id reported twice"
    assert rh.n_live == ro.n_live
    assert rh.pseudo_roots == ro.pseudo_roots
    assert rh.sup_edges == ro.sup_edges
    assert rh.edges_scanned == ro.edges_scanned


@pytest.fixture
def sharded(hip_mod):
    made = []

    def make(G, **kw):
        g = hip_mod.ShardedShadowGraph(G, **kw)
        made.append(g)
        return g
    yield make
    for g in made:
        g.close()


def test_shard_of_partitions_ids(hip_mod):
    ids = np.arange(1, 20001, dtype=np.uint64) | np.uint64(1 << 48)
    for G in (2, 3, 8):
        homes = [hip_mod.shard_of(int(i), G) for i in ids]
        counts = np.bincount(homes, minlength=G)
        assert counts.min() > 0.8 * len(ids) / G  # balanced
    assert hip_mod.shard_of(12345, 1) == 0


@pytest.mark.parametrize("G", [2, 3])
@pytest.mark.parametrize("name", sorted(kats.SCENARIOS))
def test_kat_scenarios_sharded(sharded, name, G):
    kats.run_scenario(sharded(G), kats.SCENARIOS[name]())


@pytest.mark.parametrize("G,split", [(2, False), (4, True)])
def test_random_spec_sharded_matches_oracle_every_wakeup(sharded, oracle_mod, G, split):
    w = kats.RandomWorld(seed=7, max_actors=600, wake_every=13)
    h, o = sharded(G), oracle_mod.OracleGraph()
    for batch in w.steps():
        h.merge_entries(batch, split=split)
        o.merge_entries(batch)
        assert h.export() == o.export()
        rh, ro = h.trace(True), o.trace(True)
        _same(rh, ro)
        w.kill(ro.kill_set())
    assert h.total_actors_seen() == o.total_actors_seen()
    assert h.live_count() == 1


@pytest.mark.parametrize("xbits,xlevels", [("1", "0"), ("2", "0"), ("1", "1"), ("2", "2")])
@pytest.mark.parametrize("G,seed,cap", [(2, 11, 0), (3, 12, 0), (4, 13, 64)])
def test_fuzz_sharded(sharded, oracle_mod, G, seed, cap, xbits, xlevels, monkeypatch):
    # CRGC_XBITS=2: every resolved mark travels in a home-slot bitmap; cap 64
    # rebuilds the shards often (both slot regions), so cached home slots go
    # stale and re-resolve; CRGC_XLEVELS=k: every mark round runs at most k
    # levels, its pending candidates carried into the next round
    monkeypatch.setenv("CRGC_XBITS", xbits)
    monkeypatch.setenv("CRGC_XLEVELS", xlevels)
    h, o = sharded(G, vertex_capacity=cap, edge_capacity=cap), oracle_mod.OracleGraph()
    fz = fuzz.Fuzz(seed)
    for step in range(14):
        eb = fz.entries(200 + 50 * step)
        h.merge_entries(eb, split=step % 2 == 0)
        o.merge_entries(eb)
        if step % 2 == 1:
            db = fz.deltas(5)
            h.merge_deltas(db); o.merge_deltas(db)
        if step == 9:
            ub = fz.undo(o.export().vertices.keys())
            h.merge_undo(ub); o.merge_undo(ub)
        assert h.export() == o.export()
        for loc in (1, 2, 3):
            assert h.count_reachable_from(loc) == o.count_reachable_from(loc)
        assert sorted(h.startWave().tolist()) == sorted(o.local_roots().tolist())
        _same(h.trace(True), o.trace(True))
        fz.sync(o.export())
    assert h.total_actors_seen() == o.total_actors_seen()
    assert h.export() == o.export()


def test_allgather_merge_form_matches_oracle(sharded, oracle_mod, monkeypatch):
    """CRGC_ROUTE=0: every shard applies its part of every shard's whole batch
    (the form above 16 shards) instead of receiving routed parts."""
    monkeypatch.setenv("CRGC_ROUTE", "0")
    h, o = sharded(3), oracle_mod.OracleGraph()
    fz = fuzz.Fuzz(17)
    for step in range(8):
        eb = fz.entries(400)
        h.merge_entries(eb, split=True)
        o.merge_entries(eb)
        assert h.export() == o.export()
        _same(h.trace(True), o.trace(True))
        fz.sync(o.export())


def test_routed_and_allgather_forms_agree(sharded, hip_mod, monkeypatch):
    """The same split batches through both merge forms give the same shards."""
    w = world.World(seed=0x5EED + 7)
    w.bulk_graph(20_000, 200_000, alpha=2.1, n_roots=200)
    batches = list(w.batches(1 << 16)) + [w.wakeup_batch(5_000) for _ in range(2)]
    routed = sharded(4)
    monkeypatch.setenv("CRGC_ROUTE", "0")
    gathered = sharded(4)
    for b in batches:
        routed.merge_entries(b, split=True)
        gathered.merge_entries(b, split=True)
    for a, c in zip(routed.shards, gathered.shards):
        assert a.export() == c.export()
    _same(routed.trace(True), gathered.trace(True))


def test_malformed_offsets_fail_every_shard(sharded):
    """A device batch whose offsets run backwards, contributed by one shard,
    is refused by every shard (the sender's route count flags it)."""
    from crgc_hip import EntryBatch
    h = sharded(2)
    a, b = (1 << 48) | 5, (1 << 48) | 6
    u8, i16, u32, u64 = np.uint8, np.int16, np.uint32, np.uint64
    bad = EntryBatch(np.array([a, b], u64), np.zeros(2, i16), np.array([2, 0], u8),
                     np.array([0, 2, 1], u32), np.array([a, a], u64), np.array([b, b], u64),
                     np.zeros(3, u32), np.zeros(0, u64), np.zeros(3, u32), np.zeros(0, u64),
                     np.zeros(0, i16)).to_device()
    empty = EntryBatch.from_entries([]).to_device()
    codes = []

    def go(s, batch):
        try:
            s.merge_entries(batch)
        except abi.CrgcError as e:
            codes.append(e.code)
    h._all(go, [(bad,), (empty,)])
    assert codes == [abi.E_INVAL, abi.E_INVAL]


def test_power_law_c1_sharded(sharded, oracle_mod):
    w = world.World(seed=0x5EED + 1)
    w.bulk_graph(100_000, 1_000_000, alpha=2.1, n_roots=1000)
    h, o = sharded(4), oracle_mod.OracleGraph()
    for b in w.batches(1 << 18):
        h.merge_entries(b, split=True)
        o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    for _ in range(3):
        b = w.wakeup_batch(10_000)
        h.merge_entries(b, split=True)
        o.merge_entries(b)
        rh = h.trace(True)
        _same(rh, o.trace(True))
        assert rh.rounds >= 2  # marks crossed shards
    assert h.export() == o.export()
    assert h.total_actors_seen() == o.total_actors_seen()


@pytest.mark.parametrize("supbin", ["1", "0"])
def test_power_law_sharded_binned_level0(sharded, oracle_mod, monkeypatch, supbin):
    """Level 0 binned in every shard (CRGC_BIN_MIN_SLOTS=0): the bins cover the
    proxy region, and with CRGC_SUPBIN the pseudo-roots' supervisor pushes —
    proxies among them — go through the bins too; host batches make the bins'
    slot bound an upper bound."""
    monkeypatch.setenv("CRGC_BIN_MIN_SLOTS", "0")
    monkeypatch.setenv("CRGC_SUPBIN", supbin)
    w = world.World(seed=0x5EED + 21)
    w.bulk_graph(60_000, 600_000, alpha=2.1, n_roots=600)
    h, o = sharded(3), oracle_mod.OracleGraph()
    for b in w.batches(1 << 18):
        h.merge_entries(b, split=True)
        o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    for _ in range(3):
        b = w.wakeup_batch(6_000)
        h.merge_entries(b, split=True)
        o.merge_entries(b)
        _same(h.trace(True), o.trace(True))
    assert h.export() == o.export()


def test_c3_chains_sharded(sharded, oracle_mod):
    w = world.World(seed=0x5EED + 3)
    w.chain_graph(n_chains=5, chain_len=300, n_sup_chains=3, sup_depth=100,
                  n_rings=10, ring_len=40)
    h, o = sharded(2), oracle_mod.OracleGraph()
    for b in w.batches(50_000):
        h.merge_entries(b)
        o.merge_entries(b)
    rh, ro = h.trace(True), o.trace(True)
    _same(rh, ro)
    assert len(ro.garbage) == 10 * 40
    assert h.export() == o.export()
    _same(h.trace(True), o.trace(True))


def test_c5_cluster_deltas_and_undo_sharded(sharded, oracle_mod):
    cw = cluster.ClusterWorld(seed=9, n_nodes=8, max_actors=2000)
    h, o = sharded(2), oracle_mod.OracleGraph()
    merged = []
    for _ in range(6):
        cw.run_turns(400)
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
    log = cw.undo_log(7, merged).to_batch(restrict_to=set(o.export().vertices))
    h.merge_undo(log)
    o.merge_undo(log)
    assert h.export() == o.export()
    assert h.count_reachable_from(8) == o.count_reachable_from(8)
    _same(h.trace(True), o.trace(True))


def test_npe_and_cme_are_collective(sharded, oracle_mod):
    from crgc_hip import Entry, EntryBatch, UndoBatch
    h = sharded(2)
    a = (1 << 48) | 77
    h.merge_entries(EntryBatch.from_entries([Entry(self=a)]))
    with pytest.raises(abi.CrgcError) as e:
        h.trace(True)
    assert e.value.code == abi.E_NULL_SUPERVISOR
    h2 = sharded(2)
    r = (1 << 48) | 1
    h2.merge_entries(EntryBatch.from_entries(
        [Entry(self=r, isRoot=True, createdOwners=[r], createdTargets=[r])]))
    before = h2.export()
    with pytest.raises(abi.CrgcError) as e:
        h2.merge_undo(UndoBatch.from_fields(3, [(r, 1, [((3 << 48) | 9, 1)])]))
    assert e.value.code == abi.E_UNDO_NEW_SHADOW
    assert h2.export() == before


def test_device_resident_batches_sharded(sharded, oracle_mod):
    w = kats.RandomWorld(seed=3, max_actors=300, wake_every=17)
    h, o = sharded(3), oracle_mod.OracleGraph()
    for batch in w.steps():
        parts = batch.split(3)
        h._all(lambda s, b: s.merge_entries(b.to_device()), [(p,) for p in parts])
        o.merge_entries(batch)
        _same(h.trace(True), o.trace(True))


def test_one_shard_protocol_matches_oracle(sharded, oracle_mod):
    """G = 1 with a transport runs every collective step of the sharded protocol."""
    h, o = sharded(1), oracle_mod.OracleGraph()
    fz = fuzz.Fuzz(21)
    for step in range(8):
        eb = fz.entries(300)
        h.merge_entries(eb); o.merge_entries(eb)
        if step % 2:
            db = fz.deltas(4)
            h.merge_deltas(db); o.merge_deltas(db)
        assert h.export() == o.export()
        _same(h.trace(True), o.trace(True))
        fz.sync(o.export())


def test_rccl_transport_single_rank(hip_mod, oracle_mod):
    """The RCCL transport (ncclCommInitRank, ncclAllGather, grouped send/recv
    around the self copy) on a one-rank communicator: RCCL refuses two ranks
    on one GPU, and the test box has one.  The 2/4/8-rank exchange is the same
    code with peers (covered by the in-process transport above)."""
    uid = hip_mod.Transport.rccl_unique_id()
    t = hip_mod.Transport.rccl(uid, 1, 0, 0)
    try:
        h = hip_mod.ShadowGraph(n_shards=1, shard=0, transport=t)
        o = oracle_mod.OracleGraph()
        w = kats.RandomWorld(seed=5, max_actors=300, wake_every=11)
        for batch in w.steps():
            h.merge_entries(batch)
            o.merge_entries(batch)
            rh, ro = h.trace(True), o.trace(True)
            _same(rh, ro)
            w.kill(ro.kill_set())
        assert h.export() == o.export()
        h.close()
    finally:
        t.close()


@pytest.mark.parametrize("xbits,xlevels,ratio,xfilter", [("0", "0", "32", "1"), ("1", "0", "32", "1"),
                                                         ("1", "0", "32", "0"), ("1", "0", "1", "1"),
                                                         ("2", "0", "32", "1"), ("1", "1", "32", "1"),
                                                         ("1", "3", "32", "1")])
def test_c4_shape_eight_shards(sharded, oracle_mod, xbits, xlevels, ratio, xfilter, monkeypatch):
    """G = 8 logical shards (the 8-GPU layout of C4) on a scaled C2/C4-shaped
    power-law graph with §8d wakeups (9 % busy, 1 % in flight), split batches:
    bit-exact against the unsharded oracle at every wakeup, with marks sent as
    ids only (0), as home-slot lists (1; with CRGC_XBITMAP_RATIO=1 as a bitmap
    wherever that is smaller), or as bitmaps (2), and rounds run to each shard's
    local fixpoint (XLEVELS 0) or capped at 1 / 3 levels; CRGC_XFILTER=0 sends
    marks whose homes are already marked too (no replicated home bitmaps)."""
    monkeypatch.setenv("CRGC_XBITS", xbits)
    monkeypatch.setenv("CRGC_XLEVELS", xlevels)
    monkeypatch.setenv("CRGC_XBITMAP_RATIO", ratio)
    monkeypatch.setenv("CRGC_XFILTER", xfilter)
    V = 200_000
    w = world.World(seed=0x5EED + 4)
    w.bulk_graph(V, 10 * V, alpha=2.1, n_roots=V // 1000, cap=100000)
    h, o = sharded(8), oracle_mod.OracleGraph()
    for b in w.batches(1 << 18):
        h.merge_entries(b, split=True)
        o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    for _ in range(3):
        b = w.wakeup(V // 10, busy=V * 9 // 100, pending=V // 100)
        h.merge_entries(b, split=True)
        o.merge_entries(b)
        rh = h.trace(True)
        _same(rh, o.trace(True))
        assert rh.rounds >= 2 and rh.ids_sent > 0  # marks crossed shards
        if xbits == "0":
            assert rh.exchange_bytes == 8 * rh.ids_sent  # ids only
        elif xlevels == "0" and xfilter == "0":  # resolved by the first trace: marks go as slots / bitmaps
            assert rh.exchange_bytes < 8 * rh.ids_sent
        # (capped rounds reach the replicated closure, whose all-gathers of the
        # graph's structure count in exchange_bytes too)
    assert h.export() == o.export()
    assert h.total_actors_seen() == o.total_actors_seen()


@pytest.mark.parametrize("xq,ratio", [("1", "32"), ("8", "32"), ("8", "1")])
def test_c4_shape_eight_shards_xscan_units(sharded, oracle_mod, xq, ratio, monkeypatch):
    """The export scan (k_xscan) with a wave per whole proxy block (1) or per
    eighth of one (8; by default a quarter, fewer units on large proxy regions), as lists and as bitmaps
    (CRGC_XBITMAP_RATIO=1): bit-exact against the unsharded oracle on G = 8."""
    monkeypatch.setenv("CRGC_XSCAN_Q", xq)
    monkeypatch.setenv("CRGC_XBITMAP_RATIO", ratio)
    V = 200_000
    w = world.World(seed=0x5EED + 5)
    w.bulk_graph(V, 10 * V, alpha=2.1, n_roots=V // 1000, cap=100000)
    h, o = sharded(8), oracle_mod.OracleGraph()
    for b in w.batches(1 << 18):
        h.merge_entries(b, split=True)
        o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    for _ in range(3):
        b = w.wakeup(V // 10, busy=V * 9 // 100, pending=V // 100)
        h.merge_entries(b, split=True)
        o.merge_entries(b)
        rh = h.trace(True)
        _same(rh, o.trace(True))
        assert rh.rounds >= 2 and rh.ids_sent > 0
    assert h.export() == o.export()


@pytest.mark.parametrize("walk", [{"CRGC_WALK": "1"},
                                  {"CRGC_WALK": "1", "CRGC_WALK_START": "64", "CRGC_WALK_MAX": "128"},
                                  {"CRGC_WALK": "1", "CRGC_WALK_START": "65536", "CRGC_WALK_MAX": "65536"},
                                  # k_tail (no k_walk) bounded by edge volume: tiny bounds, so
                                  # takeovers are refused or bail at their first hubs (round 6)
                                  {"CRGC_TAIL_EDGES": "64"},
                                  {"CRGC_TAIL_EDGES": "512", "CRGC_TAIL_START": "65536",
                                   "CRGC_TAIL_MAX": "65536"}])
def test_c4_shape_eight_shards_walk_forms(sharded, oracle_mod, walk, monkeypatch):
    """A mark round's narrow levels by k_walk (WALK_WG workgroups with grid
    barriers; off by default, the level kernels and k_tail run them): at its
    default thresholds, taking over early and bailing often (64 / 128), or
    taking every listed level up to its queue's capacity — bit-exact against
    the unsharded oracle (G = 8, C4-shaped)."""
    for k, v in walk.items():
        monkeypatch.setenv(k, v)
    V = 100_000
    w = world.World(seed=0x5EED + 14)
    w.bulk_graph(V, 10 * V, alpha=2.1, n_roots=V // 1000, cap=100000)
    h, o = sharded(8), oracle_mod.OracleGraph()
    for b in w.batches(1 << 18):
        h.merge_entries(b, split=True)
        o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    for _ in range(2):
        b = w.wakeup(V // 10, busy=V * 9 // 100, pending=V // 100)
        h.merge_entries(b, split=True)
        o.merge_entries(b)
        _same(h.trace(True), o.trace(True))
    assert h.export() == o.export()


def test_forty_shards_rebuild_homes_above_32(sharded, oracle_mod):
    """Home-slot generations of shards >= 32 (the per-home mask is
    64 bits wide).  Shards 33, 35 and 39 compact between traces, renumbering
    their slots; every other shard's proxies of them must forget their cached
    home slots (and only those), or marks land on renumbered shadows."""
    G = 40
    h, o = sharded(G, vertex_capacity=64, edge_capacity=64), oracle_mod.OracleGraph()
    fz = fuzz.Fuzz(41)
    for step in range(6):
        eb = fz.entries(800)
        h.merge_entries(eb, split=True)
        o.merge_entries(eb)
        if step >= 1:
            for r in (33, 35, 39):
                h.shards[r].compact()  # local: bumps shard r's slot generation only
        assert h.export() == o.export()
        rh, ro = h.trace(True), o.trace(True)
        _same(rh, ro)
        if step >= 1:
            assert rh.rounds >= 2
        fz.sync(o.export())
    assert h.export() == o.export()


@pytest.mark.parametrize("G,seed", [(2, 31), (3, 32), (8, 33)])
def test_fuzz_sharded_closure(sharded, oracle_mod, G, seed, monkeypatch):
    """The replicated chain closure (crgc_xchain.hip) forced from the first
    round of every mark (it normally takes over deep, narrow marks after 8
    rounds): branching shadows, halted shadows (undo logs), proxies of
    collected actors, supervisors across shards, investigate mode."""
    monkeypatch.setenv("CRGC_XCLOSURE_AFTER", "1")
    monkeypatch.setenv("CRGC_XCLOSURE_NARROW", "0")
    h, o = sharded(G), oracle_mod.OracleGraph()
    fz = fuzz.Fuzz(seed)
    for step in range(12):
        eb = fz.entries(300 + 60 * step)
        h.merge_entries(eb, split=step % 2 == 0)
        o.merge_entries(eb)
        if step % 2 == 1:
            db = fz.deltas(5)
            h.merge_deltas(db); o.merge_deltas(db)
        if step == 7:
            ub = fz.undo(o.export().vertices.keys())
            h.merge_undo(ub); o.merge_undo(ub)
        assert h.export() == o.export()
        for loc in (1, 2, 3):
            assert h.count_reachable_from(loc) == o.count_reachable_from(loc)
        _same(h.trace(True), o.trace(True))
        fz.sync(o.export())
    assert h.export() == o.export()


def test_c4_shape_eight_shards_closure(sharded, oracle_mod, monkeypatch):
    """The closure forced on the G = 8 C4-shaped power-law graph: wide marks,
    many branching shadows, supervisor chains across shards."""
    monkeypatch.setenv("CRGC_XCLOSURE_AFTER", "1")
    monkeypatch.setenv("CRGC_XCLOSURE_NARROW", "0")
    V = 100_000
    w = world.World(seed=0x5EED + 4)
    w.bulk_graph(V, 10 * V, alpha=2.1, n_roots=V // 1000, cap=100000)
    h, o = sharded(8), oracle_mod.OracleGraph()
    for b in w.batches(1 << 18):
        h.merge_entries(b, split=True)
        o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    for _ in range(2):
        b = w.wakeup(V // 10, busy=V * 9 // 100, pending=V // 100)
        h.merge_entries(b, split=True)
        o.merge_entries(b)
        _same(h.trace(True), o.trace(True))
    assert h.export() == o.export()


def test_rebuild_keeps_every_proxy_before_any_trace(sharded, oracle_mod, capfd, monkeypatch):
    """A sharded load that outgrows its capacity before the first trace: every
    shard's alive slots are mostly proxies (the far ends of its edges, in the
    proxy region since round 5), far more than the home shadows it created.  The
    rebuild must size both new regions from the alive slots (crgc_api.hip
    rebuild: counted on the device), not from the homes created since the last
    trace — round 4's C4 over 8 logical shards put 68 M alive slots into 27 M
    and its passes wrote past the new arrays.  Sets and counts must equal the
    oracle's."""
    monkeypatch.setenv("CRGC_LEVEL_LOG", "1")
    w = world.World(seed=0x5EED + 44)
    w.bulk_graph(200_000, 2_000_000, alpha=2.1, n_roots=200)
    h, o = sharded(8, vertex_capacity=4096, edge_capacity=32768), oracle_mod.OracleGraph()
    for b in w.batches(1 << 13):
        h.merge_entries(b, split=True)
        o.merge_entries(b)
    rh, ro = h.trace(True), o.trace(True)
    _same(rh, ro)
    err = capfd.readouterr().err
    lines = [line for line in err.splitlines() if line.startswith("[crgc] rebuild:")]
    assert lines, "the load was meant to outgrow the first capacity"
    homes = [int(line.split("(alive ")[1].split(")")[0]) for line in lines]
    proxies = [int(line.split("(alive ")[2].split(")")[0]) for line in lines]
    assert max(homes) <= 30_000          # homes ~25 k per shard
    assert max(proxies) > 2 * max(homes)  # the proxies dominate (~90 k)
    b = w.wakeup(20_000, busy=18_000, pending=2_000)
    h.merge_entries(b, split=True)
    o.merge_entries(b)
    _same(h.trace(True), o.trace(True))
    assert h.export() == o.export()
