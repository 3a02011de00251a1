"""Streams that drive Java `int` fields past +-2^31.

ShadowGraph keeps Shadow.recvCount and the outgoing counts as Java ints
(Shadow.java:13-27), updated by `+=` / `-=` in mergeEntry (:77-123),
mergeDelta (:138, :150-154) and mergeUndoLog (:166-172): two's-complement
wraparound.  Each stream is a list of ("entries" | "deltas" | "undo", batch)
steps followed by traces; the expected values follow from 32-bit wrapping
arithmetic and are asserted against the exported graph.
"""
import numpy as np

from crgc_hip import Entry, EntryBatch, DeltaBatch, UndoBatch, abi

LOC = 1
INT_MAX = 2**31 - 1


def aid(k: int) -> int:
    return (LOC << 48) | (0x1000 + k)


def wrap(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - 2**32 if x & 0x80000000 else x


ROOT, A, B, C = aid(0), aid(1), aid(2), aid(3)


def setup_batch() -> EntryBatch:
    """Root R spawns A, B, C and keeps refs to them (A, B, C local, supervised)."""
    es = [Entry(self=ROOT, isRoot=True, createdOwners=[ROOT], createdTargets=[ROOT],
                spawnedActors=[A, B, C])]
    for x in (A, B, C):
        es.append(Entry(self=x, createdOwners=[x, ROOT], createdTargets=[x, x]))
    return EntryBatch.from_entries(es)


def recv_entries(actor: int, n: int, per: int = 32767) -> EntryBatch:
    """n entries of `actor`, each reporting `per` received messages (the
    per-entry cap of State.recordMessageReceived, CRGC.scala:121-122)."""
    return EntryBatch.from_entries([Entry(self=actor, recvCount=per, isBusy=True) for _ in range(n)])


def delta(rows) -> DeltaBatch:
    return DeltaBatch.from_rows(rows)


def streams():
    """name -> (steps, expectations); expectations: {actor: recv} and {(o, t): count}."""
    out = {}
    # 1. recv through entries: 65538 x 32767 crosses INT_MAX
    n = 65538
    out["entries_recv"] = ([("entries", setup_batch()), ("entries", recv_entries(A, n))],
                           {A: wrap(n * 32767)}, {})
    # 2. recv and an edge count through delta shadows (int32 fields, DeltaShadow.java:11-51)
    nd = abi.DELTA_INTERNED
    rows1 = [(B, INT_MAX, abi.NO_ACTOR, nd, [(C, INT_MAX)])]
    rows2 = [(B, 5, abi.NO_ACTOR, nd, [(C, 3)])]
    out["deltas_recv_and_count"] = (
        [("entries", setup_batch()), ("deltas", delta(rows1)), ("deltas", delta(rows2))],
        {B: wrap(INT_MAX + 5)}, {(B, C): wrap(INT_MAX + 3)})
    # 3. a count that wraps back to exactly 0 is absent (updateOutgoing deletes it, :64-73)
    rows3 = [(A, 0, abi.NO_ACTOR, nd, [(C, -(2**31))])]
    rows4 = [(A, 0, abi.NO_ACTOR, nd, [(C, -(2**31))])]
    out["count_wraps_to_zero"] = (
        [("entries", setup_batch()), ("deltas", delta(rows3)), ("deltas", delta(rows4))],
        {}, {(A, C): 0})
    # 4. undo-log fields (UndoLog.Field.messageCount / createdRefs, int)
    log = UndoBatch.from_fields(7, [(C, INT_MAX, [(A, INT_MAX)]), (A, 2, [(C, 2)])])
    pre = [(C, 9, abi.NO_ACTOR, nd, [(A, 9)])]
    out["undo_fields"] = (
        [("entries", setup_batch()), ("deltas", delta(pre)), ("undo", log)],
        {C: wrap(9 + INT_MAX), A: 2}, {(C, A): wrap(9 + INT_MAX), (A, C): 2})
    # 5. entries' send counts subtracted below INT_MIN: recv starts at -2^31 + 5
    rows5 = [(B, -(2**31) + 5, abi.NO_ACTOR, nd, [])]
    ents = EntryBatch.from_entries([Entry(self=ROOT, isRoot=True, updatedRefs=[B], updatedInfos=[2 * 16383])] * 3)
    out["entries_send_underflow"] = (
        [("entries", setup_batch()), ("deltas", delta(rows5)), ("entries", ents)],
        {B: wrap(-(2**31) + 5 - 3 * 16383)}, {})
    return out


def apply(g, steps):
    for kind, b in steps:
        if kind == "entries":
            g.merge_entries(b)
        elif kind == "deltas":
            g.merge_deltas(b)
        else:
            g.merge_undo(b)


def check(state, exp_recv, exp_edges):
    for a, v in exp_recv.items():
        assert state.vertices[a][0] == v, (hex(a), state.vertices[a][0], v)
    for (o, t), c in exp_edges.items():
        assert state.edges.get((o, t), 0) == c, (hex(o), hex(t), state.edges.get((o, t)), c)
