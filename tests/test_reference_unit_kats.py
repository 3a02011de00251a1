"""The reference's unit specs, restated against the host-side mirrors (CPU).

* RefobInfoSpec.scala:10-60 — the 16-bit info word under random increments,
  resets and a final deactivation.
* SerializationSpec.scala:12-53 — DeltaShadow wire sizes 25 and 13 bytes and
  round trips; :80-98 — a DeltaGraph built from one entry has size 2.
"""
import random

import pytest

from crgc_hip.batch import RefobInfo
from delta import DeltaGraph, DeltaShadow, UndoLog, IngressEntry, deltas_from_entries
from mutator import Mutator


@pytest.mark.parametrize("seed", range(20))
def test_refob_info_property(seed):
    rng = random.Random(seed)
    incs, resets = rng.randint(0, 1000), rng.randint(0, 1000)
    ops = ["inc"] * incs + ["reset"] * resets
    rng.shuffle(ops)
    ops.append("deactivate")
    real_active, real_count = True, 0
    info = RefobInfo.activeRefob
    assert RefobInfo.isActive(info) and RefobInfo.count(info) == 0
    for op in ops:
        if op == "inc":
            real_count += 1
            info = RefobInfo.incSendCount(info)
        elif op == "reset":
            real_count = 0
            info = RefobInfo.resetCount(info)
        else:
            real_active = False
            info = RefobInfo.deactivate(info)
        if real_count <= 16383:  # RefobInfo.canIncrement bound (CRGC flushes before it)
            assert RefobInfo.isActive(info) == real_active
            assert RefobInfo.count(info) == real_count


def test_delta_shadow_serialization_test1():
    s = DeltaShadow()
    s.recvCount, s.supervisor, s.interned, s.isRoot, s.isBusy = 1, 2, True, False, True
    s.outgoing[1] = 2
    s.outgoing[3] = 4
    b = s.serialize()
    assert len(b) == 25
    t = DeltaShadow.deserialize(b)
    assert (t.recvCount, t.supervisor, t.interned, t.isRoot, t.isBusy, t.outgoing) == \
        (1, 2, True, False, True, {1: 2, 3: 4})


def test_delta_shadow_serialization_test2():
    s = DeltaShadow()
    s.recvCount, s.supervisor, s.interned, s.isRoot, s.isBusy = 2, 0, False, True, False
    b = s.serialize()
    assert len(b) == 13
    t = DeltaShadow.deserialize(b)
    assert (t.recvCount, t.supervisor, t.interned, t.isRoot, t.isBusy, t.outgoing) == \
        (2, 0, False, True, False, {})


def test_delta_graph_two_actor_graph_has_size_two():
    m = Mutator()
    st1 = m.initState(None, actor_id=(1 << 48) | 1)
    st1.created = []  # SerializationSpec builds State directly: no init records
    from mutator import Refob
    refob2 = Refob((1 << 48) | 2)
    st1.recordNewActor(refob2)
    refob2.info = RefobInfo.incSendCount(refob2.info)
    st1.recordUpdatedRefob(refob2)
    entry = st1.flushToEntry(False)
    g = DeltaGraph(address=1)
    g.mergeEntry(entry)
    assert g.size == 2


def test_delta_graph_full_rule_and_undo_log():
    # DeltaGraph.isFull (DeltaGraph.java:174-180) cuts graphs at size + 4F + 1 >= 64.
    m = Mutator(location=2)
    root = m.spawn_root()
    for _ in range(120):
        ref, child = m.spawn(root)
        m.onBlock(child)
    m.onBlock(root)
    graphs = deltas_from_entries(m.queue, address=2)
    assert len(graphs) > 1 and all(g.size < 64 for g in graphs)
    log = UndoLog(2)
    for g in graphs:
        log.mergeDeltaGraph(g)
    ing = IngressEntry(egress=2, ingress=1)
    ing.isFinal = True
    log.mergeIngressEntry(ing)
    assert log.finalizedBy == {1}
