"""Host-side DeltaGraph / UndoLog / IngressEntry builders (cluster-mode inputs).

In the reference these stay on the JVM: every
node compresses its entry stream into DeltaGraphs broadcast to the other
collectors (LocalGC.scala:159-177, 191-196), and a downed node's effects are
undone from an UndoLog built from its deltas and the survivors' ingress
entries (UndoLog.java:39-93).  They are restated here to generate the C5
cluster stream; `to_batch()` decodes the compressed ids (DeltaGraph.decoder,
DeltaGraph.java:162-169) into the crgc_delta_batch the C ABI takes.

  DeltaShadow        DeltaShadow.java:11-84 (wire format pinned by
                     SerializationSpec.scala:12-53: 13 + 6 bytes per outgoing)
  DeltaGraph         DeltaGraph.java:60-187
  IngressEntry       IngressEntry.java:12-100 (admission counting)
  UndoLog            UndoLog.java:16-104
"""
from __future__ import annotations

import os
import struct
import sys
from typing import Dict, List, Optional

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "uigc-akka_amd"))
from crgc_hip import abi  # noqa: E402
from crgc_hip.batch import DeltaBatch, Entry, RefobInfo, UndoBatch  # noqa: E402


def _update(m: dict, key, delta: int):
    """updateOutgoing: absent == 0, zero deletes the key (DeltaGraph.java:127-136)."""
    c = m.get(key, 0) + delta
    if c == 0:
        m.pop(key, None)
    else:
        m[key] = c


class DeltaShadow:
    def __init__(self):
        self.outgoing: Dict[int, int] = {}
        self.recvCount = 0
        self.supervisor = -1
        self.interned = False
        self.isRoot = False
        self.isBusy = False

    def serialize(self) -> bytes:
        """DataOutput big-endian layout of DeltaShadow.serialize (DeltaShadow.java:57-69)."""
        out = struct.pack(">ih???i", self.recvCount, self.supervisor, self.interned,
                          self.isRoot, self.isBusy, len(self.outgoing))
        for k, v in self.outgoing.items():
            out += struct.pack(">hi", k, v)
        return out

    @staticmethod
    def deserialize(buf: bytes) -> "DeltaShadow":
        d = DeltaShadow()
        d.recvCount, d.supervisor, d.interned, d.isRoot, d.isBusy, n = \
            struct.unpack_from(">ih???i", buf, 0)
        off = 13
        for _ in range(n):
            k, v = struct.unpack_from(">hi", buf, off)
            d.outgoing[k] = v
            off += 6
        return d


class DeltaGraph:
    def __init__(self, address: int, entry_field_size: int = 4, delta_graph_size: int = 64):
        self.address = address
        self.F = entry_field_size
        self.capacity = delta_graph_size
        self.compressionTable: Dict[int, int] = {}
        self.shadows: List[DeltaShadow] = []

    @property
    def size(self) -> int:
        return len(self.shadows)

    def encode(self, ref: int) -> int:
        i = self.compressionTable.get(ref)
        if i is not None:
            return i
        i = len(self.shadows)
        self.compressionTable[ref] = i
        self.shadows.append(DeltaShadow())
        return i

    def mergeEntry(self, e: Entry):  # DeltaGraph.java:73-125
        me = self.encode(e.self)
        s = self.shadows[me]
        s.interned = True
        s.recvCount += e.recvCount
        s.isBusy = e.isBusy
        s.isRoot = e.isRoot
        for owner, target in zip(e.createdOwners, e.createdTargets):
            t = self.encode(target)
            o = self.encode(owner)
            _update(self.shadows[o].outgoing, t, 1)
        for child in e.spawnedActors:
            self.shadows[self.encode(child)].supervisor = me
        for ref, info in zip(e.updatedRefs, e.updatedInfos):
            t = self.encode(ref)
            cnt = RefobInfo.count(info)
            if cnt > 0:
                self.shadows[t].recvCount -= cnt
            if not RefobInfo.isActive(info):
                _update(s.outgoing, t, -1)

    def isFull(self) -> bool:  # DeltaGraph.java:174-180
        return self.size + 4 * self.F + 1 >= self.capacity

    def nonEmpty(self) -> bool:
        return self.size > 0

    def decoder(self) -> List[int]:
        refs = [0] * self.size
        for ref, i in self.compressionTable.items():
            refs[i] = ref
        return refs

    def rows(self):
        dec = self.decoder()
        out = []
        for i, s in enumerate(self.shadows):
            fl = (abi.DELTA_INTERNED if s.interned else 0) | \
                 (abi.DELTA_ROOT if s.isRoot else 0) | (abi.DELTA_BUSY if s.isBusy else 0)
            sup = dec[s.supervisor] if s.supervisor >= 0 else abi.NO_ACTOR
            out.append((dec[i], s.recvCount, sup, fl, [(dec[k], v) for k, v in s.outgoing.items()]))
        return out

    def to_batch(self) -> DeltaBatch:
        return DeltaBatch.from_rows(self.rows())


def deltas_from_entries(entries, address, F=4, dgs=64) -> List[DeltaGraph]:
    """LocalGC's Wakeup loop for num-nodes > 1 (LocalGC.scala:159-177)."""
    out, g = [], DeltaGraph(address, F, dgs)
    for e in entries:
        g.mergeEntry(e)
        if g.isFull():
            out.append(g)
            g = DeltaGraph(address, F, dgs)
    if g.nonEmpty():
        out.append(g)
    return out


class IngressField:
    def __init__(self):
        self.messageCount = 0
        self.createdRefs: Dict[int, int] = {}


class IngressEntry:
    """Messages from `egressAddress` admitted at `ingressAddress` (IngressEntry.java)."""

    def __init__(self, egress: int, ingress: int):
        self.egressAddress = egress
        self.ingressAddress = ingress
        self.admitted: Dict[int, IngressField] = {}
        self.isFinal = False

    def onMessage(self, recipient: int, ref_targets):  # IngressEntry.java:91-100
        f = self.admitted.setdefault(recipient, IngressField())
        f.messageCount += 1
        for t in ref_targets:
            f.createdRefs[t] = f.createdRefs.get(t, 0) + 1


class UndoLog:
    def __init__(self, nodeAddress: int):
        self.nodeAddress = nodeAddress
        self.finalizedBy = set()
        self.admitted: Dict[int, IngressField] = {}

    def mergeDeltaGraph(self, delta: DeltaGraph):  # UndoLog.java:39-67
        dec = delta.decoder()
        for i, s in enumerate(delta.shadows):
            if s.interned:
                continue
            f = self.admitted.setdefault(dec[i], IngressField())
            f.messageCount -= s.recvCount
            for k, v in s.outgoing.items():
                _update(f.createdRefs, dec[k], -v)

    def mergeIngressEntry(self, entry: IngressEntry):  # UndoLog.java:69-93
        for actor, ef in entry.admitted.items():
            f = self.admitted.setdefault(actor, IngressField())
            f.messageCount += ef.messageCount
            for t, c in ef.createdRefs.items():
                _update(f.createdRefs, t, c)
        if entry.isFinal:
            self.finalizedBy.add(entry.ingressAddress)

    def to_batch(self, restrict_to: Optional[set] = None) -> UndoBatch:
        fields = []
        for a, f in self.admitted.items():
            refs = [(t, c) for t, c in f.createdRefs.items()
                    if restrict_to is None or t in restrict_to]
            fields.append((a, f.messageCount, refs))
        return UndoBatch.from_fields(self.nodeAddress, fields)
