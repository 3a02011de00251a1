"""The DeltaGraph production oracle (oracle/deltagraph.py), on CPU.

Pinned by the reference's SerializationSpec.scala (DeltaShadow wire sizes 25
and 13 bytes, :12-67; a DeltaGraph from one two-actor entry has size 2,
:80-98), by OpenJDK HashMap iteration facts, and against the independent
restatements used to generate the C5 streams (workload/delta.py and
workload/deltas.cpp): same graph cuts, same shadows, same outgoing maps.
"""
import struct

import numpy as np
import pytest

import deltagraph as dgo
import delta
import fuzz
import kats
import world
from crgc_hip import Entry, EntryBatch, RefobInfo


def test_delta_shadow_wire_sizes_pinned_by_serialization_spec():
    s = dgo.DeltaShadow()  # SerializationSpec.scala:12-25
    s.recvCount, s.supervisor, s.interned, s.isRoot, s.isBusy = 1, 2, True, False, True
    s.outgoing.put(1, 2)
    s.outgoing.put(3, 4)
    b = s.serialize()
    assert len(b) == 25
    assert struct.unpack(">ih???ihihi", b) == (1, 2, True, False, True, 2, 1, 2, 3, 4)
    s2 = dgo.DeltaShadow()  # :42-53
    s2.recvCount, s2.supervisor, s2.isRoot = 2, 0, True
    assert len(s2.serialize()) == 13


def test_two_actor_graph_size_pinned_by_serialization_spec():
    # :80-98: state1.recordNewActor(refob2); refob2.incSendCount(); recordUpdatedRefob(refob2)
    r1, r2 = (1 << 48) | 1, (1 << 48) | 2
    info = RefobInfo.incSendCount(RefobInfo.activeRefob)
    e = Entry(self=r1, spawnedActors=[r2], updatedRefs=[r2], updatedInfos=[info])
    gs = dgo.build(EntryBatch.from_entries([e]))
    assert len(gs) == 1 and gs[0].size == 2
    assert gs[0].shadows[1].recvCount == -1 and gs[0].shadows[1].supervisor == 0


def test_java_hashmap_iteration_order():
    m = dgo.JavaHashMap()
    for k in (17, 1, 33):  # one bin at 16 bins: insertion order
        m.put(k, k)
    assert [k for k, _ in m.items()] == [17, 1, 33]
    m.remove(17)
    m.put(17, 5)  # a re-put key goes to the tail of its bin
    assert [k for k, _ in m.items()] == [1, 33, 17]
    m = dgo.JavaHashMap()
    for k in [20, 4] + list(range(5, 16)):  # 13 keys: the 13th put resizes to 32 bins
        m.put(k, 1)
    assert len(m.table) == 32
    assert [k for k, _ in m.items()] == [4] + list(range(5, 16)) + [20]
    m.remove(4)
    assert len(m.table) == 32  # never shrinks


def _batches():
    w = kats.RandomWorld(seed=5, max_actors=200, wake_every=9)
    for i, b in enumerate(w.steps()):
        if i % 5 == 0:
            yield b
    fz = fuzz.Fuzz(3)
    yield fz.entries(400)
    wo = world.World(seed=11, location=2)
    wo.bulk_graph(2000, 20000, alpha=2.1, n_roots=20)
    yield wo.take(3000)
    yield wo.wakeup_batch(2000)


def _outgoing_maps(rows):
    return [(r[0], r[1], r[2], r[3], dict(r[4])) for r in rows]


def test_oracle_matches_workload_restatements():
    """Same cuts and contents as workload/delta.py (Python dicts) and
    workload/deltas.cpp; only the outgoing order (HashMap vs insertion) differs."""
    for b in _batches():
        ours = dgo.build(b)
        ref = delta.deltas_from_entries(b.to_entries(), address=1)
        assert [g.size for g in ours] == [g.size for g in ref]
        for g, r in zip(ours, ref):
            assert _outgoing_maps(g.rows()) == _outgoing_maps(r.rows())
            # same bytes up to the order of each outgoing map's entries
            assert len(g.shadows_bytes()) == 2 + sum(len(s.serialize()) for s in r.shadows[:r.size])
        d, graph_off = world.deltas_of(b)
        cols, g_off, _, _ = dgo.arrays(ours)
        assert np.array_equal(graph_off, g_off)
        for k in ("id", "recv_count", "supervisor", "flags", "out_off"):
            assert np.array_equal(getattr(d, k), cols[k]), k


@pytest.mark.parametrize("F,DGS", [(4, 64), (2, 32), (4, 20), (1, 8)])
def test_graph_cuts_follow_is_full(F, DGS):
    b = fuzz.Fuzz(9).entries(300)
    b = EntryBatch.from_entries([Entry(**{**e.__dict__,
                                          "createdOwners": e.createdOwners[:F],
                                          "createdTargets": e.createdTargets[:F],
                                          "spawnedActors": e.spawnedActors[:F],
                                          "updatedRefs": e.updatedRefs[:F],
                                          "updatedInfos": e.updatedInfos[:F]})
                                for e in b.to_entries()])
    gs = dgo.build(b, F, DGS)
    assert sum(1 for _ in gs) >= 1
    for g in gs[:-1]:
        assert g.is_full() and g.size < DGS
    assert gs[-1].size < DGS
