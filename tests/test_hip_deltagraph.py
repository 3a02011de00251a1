"""crgc_build_delta_graphs (device DeltaGraph production)
against oracle/deltagraph.py: the graph cuts, every decoded column, the
outgoing entries in java.util.HashMap order and the DataOutput bytes of
DeltaShadow.serialize, bit-exact."""
import numpy as np
import pytest

import deltagraph as dgo
import fuzz
import kats
import world
from crgc_hip import Entry, EntryBatch, RefobInfo, abi

pytestmark = pytest.mark.gpu

COLS = ("id", "recv_count", "supervisor", "flags", "out_off", "out_target", "out_count")


def _np(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


def _check(g, batch, device_in=False, device_out=False):
    F, DGS = g.F, g.DGS
    want_cols, want_goff, want_wire, want_woff = dgo.arrays(dgo.build(batch, F, DGS))
    d, goff, wire, woff = g.build_delta_graphs(batch.to_device() if device_in else batch,
                                               device_out=device_out)
    assert np.array_equal(_np(goff), want_goff)
    for k in COLS:
        assert np.array_equal(_np(getattr(d, k)).view(want_cols[k].dtype), want_cols[k]), k
    assert np.array_equal(_np(woff), want_woff)
    assert bytes(_np(wire)) == bytes(want_wire)
    return len(want_goff) - 1


def _trim(b, F):
    return EntryBatch.from_entries([Entry(**{**e.__dict__,
                                             "createdOwners": e.createdOwners[:F],
                                             "createdTargets": e.createdTargets[:F],
                                             "spawnedActors": e.spawnedActors[:F],
                                             "updatedRefs": e.updatedRefs[:F],
                                             "updatedInfos": e.updatedInfos[:F]})
                                   for e in b.to_entries()])


def test_random_spec_wakeups(hip_mod):
    g = hip_mod.ShadowGraph()
    w = kats.RandomWorld(seed=13, max_actors=400, wake_every=11)
    for i, b in enumerate(w.steps()):
        _check(g, b, device_in=i % 2 == 1, device_out=i % 3 == 2)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_entries(hip_mod, seed):
    g = hip_mod.ShadowGraph()
    fz = fuzz.Fuzz(seed)
    for n in (1, 7, 300, 2000):
        _check(g, fz.entries(n))


def test_power_law_wakeups(hip_mod):
    g = hip_mod.ShadowGraph()
    w = world.World(seed=0x5EED + 1, location=3)
    w.bulk_graph(20_000, 200_000, alpha=2.1, n_roots=200)
    assert _check(g, w.take(20_000)) > 100
    assert _check(g, w.wakeup_batch(10_000), device_in=True, device_out=True) > 100


@pytest.mark.parametrize("F,DGS", [(2, 32), (4, 20), (1, 8), (4, 64)])
def test_field_and_graph_sizes(hip_mod, F, DGS):
    g = hip_mod.ShadowGraph(entry_field_size=F, delta_graph_size=DGS)
    _check(g, _trim(fuzz.Fuzz(40 + F).entries(1500), F))


def test_long_graphs_many_messages(hip_mod):
    """ManyMessagesSpec-like wakeup (ManyMessagesSpec.scala:33-42): two actors
    trading thousands of entries never fill a graph — one graph spans the
    batch (deferred spans resolved by k_dg_long); then the same again after
    a burst of fresh actors, so the chain has long and short graphs."""
    g = hip_mod.ShadowGraph()
    a, b = (1 << 48) | 1, (1 << 48) | 2
    inc = RefobInfo.incSendCount(RefobInfo.activeRefob)
    talk = [Entry(self=a if i % 2 else b, updatedRefs=[b if i % 2 else a], updatedInfos=[inc],
                  recvCount=1) for i in range(3000)]
    assert _check(g, EntryBatch.from_entries(talk)) == 1
    burst = [Entry(self=(1 << 48) | (100 + i), spawnedActors=[(1 << 48) | (10_000 + i)])
             for i in range(200)]
    assert _check(g, EntryBatch.from_entries(talk[:700] + burst + talk[:1000] + burst[:50])) > 3


def test_graphs_with_many_outgoing_records(hip_mod):
    """More than DG_RCAP distinct (owner, target) pairs in one graph: the
    global-store pass, and resized HashMaps (more than 12 keys per owner)."""
    g = hip_mod.ShadowGraph()
    ids = [(1 << 48) | (500 + i) for i in range(30)]
    es = []
    for i in range(400):
        o = ids[i % 30]
        ts = [ids[(i // 30 * 4 + k) % 30] for k in range(4)]
        es.append(Entry(self=o, createdOwners=[o] * 4, createdTargets=ts))
        if i % 9 == 0:
            es.append(Entry(self=o, updatedRefs=ts[:2],
                            updatedInfos=[RefobInfo.deactivate(RefobInfo.activeRefob)] * 2))
    b = EntryBatch.from_entries(es)
    gs = dgo.build(b)
    assert max(sum(len(s.outgoing) for s in x.shadows) for x in gs) > 64
    assert max(len(s.outgoing.table or []) for x in gs for s in x.shadows) >= 32
    _check(g, b)
    _check(g, b, device_in=True, device_out=True)


def test_empty_and_errors(hip_mod):
    g = hip_mod.ShadowGraph()
    assert _check(g, EntryBatch.empty()) == 0
    with pytest.raises(abi.CrgcError) as e:
        hip_mod.ShadowGraph(entry_field_size=4, delta_graph_size=16).build_delta_graphs(
            fuzz.Fuzz(1).entries(10))
    assert e.value.code == abi.E_INVAL
    with pytest.raises(abi.CrgcError) as e:  # a reserved id
        g.build_delta_graphs(EntryBatch.from_entries([Entry(self=abi.NO_ACTOR)]))
    assert e.value.code == abi.E_INVAL


def test_decoded_graphs_merge_like_the_oracles(hip_mod, oracle_mod):
    """A remote node merges the device-built deltas (crgc_merge_deltas on the
    device arrays) exactly as the oracle merges its own DeltaGraphs."""
    g = hip_mod.ShadowGraph()
    remote, o = hip_mod.ShadowGraph(), oracle_mod.OracleGraph()
    w = world.World(seed=77, location=5)
    w.bulk_graph(5000, 40000, alpha=2.1, n_roots=50)
    for b in [w.take(8000), w.wakeup_batch(3000)]:
        d, _, _, _ = g.build_delta_graphs(b, device_out=True)
        remote.merge_deltas(d)
        cols, _, _, _ = dgo.arrays(dgo.build(b))
        from crgc_hip import DeltaBatch
        o.merge_deltas(DeltaBatch(*(cols[k] for k in COLS)))
        assert remote.export() == o.export()


def test_device_outputs_grow_after_a_speculative_write(hip_mod):
    """Device outputs sized by a small batch, then a larger one: the write pass
    that runs on the device's counts (before the host sees the totals) finds
    the outputs too small, writes nothing and reports E2BIG; the wrapper grows
    them and the second call's bytes are exact.  Then smaller again (the
    outputs fit: written speculatively)."""
    g = hip_mod.ShadowGraph()
    w = world.World(seed=21)
    w.bulk_graph(20_000, 200_000, alpha=2.1, n_roots=50)
    for n in (300, 20_000, 1_000):
        b = w.wakeup_batch(n)
        assert _check(g, b, device_in=True, device_out=True) > 0


@pytest.mark.parametrize("device_out", [False, True])
def test_malformed_offsets_are_rejected_without_writes(hip_mod, device_out):
    """Offsets that decrease, or run past the records, fail the call with
    E_INVAL (as the merges do); the single replay pass writes into slots bounded
    by each graph's entries, so even a malformed batch stays inside them.  The
    handle is usable afterwards."""
    g = hip_mod.ShadowGraph()
    good = fuzz.Fuzz(5).entries(600)
    for field, at, val in (("created_off", 300, 0), ("updated_off", 200, 1 << 30),
                           ("spawned_off", 599, 0)):
        arrs = {k: np.array(getattr(good, k)) for k in EntryBatch.__slots__[:11]}
        arrs[field][at] = val
        bad = EntryBatch(arrs["self"], arrs["recv_count"], arrs["flags"], arrs["created_off"],
                         arrs["created_owner"], arrs["created_target"], arrs["spawned_off"],
                         arrs["spawned"], arrs["updated_off"], arrs["updated_ref"], arrs["updated_info"])
        with pytest.raises(abi.CrgcError) as e:
            g.build_delta_graphs(bad, device_out=device_out)
        assert e.value.code == abi.E_INVAL, field
    assert _check(g, good, device_out=device_out) > 0
