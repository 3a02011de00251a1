"""CPU oracle for DeltaGraph production — TEST
INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker of crgc_build_delta_graphs, never by the
product.

Restates, entry by entry:
  LocalGC Wakeup with num-nodes > 1        LocalGC.scala:159-177
      deltaGraph.mergeEntry; finalize when isFull; finalize the non-empty rest
  DeltaGraph.mergeEntry / encode / isFull  DeltaGraph.java:73-156, 174-180
  DeltaGraph.serialize (the shadows part)  DeltaGraph.java:196-200
  DeltaShadow.serialize                    DeltaShadow.java:57-69
and the one third-party piece of arithmetic on the path, the iteration order
of DeltaShadow.outgoing, a java.util.HashMap<Short, Integer> (OpenJDK 17
java/util/HashMap.java, not in /root/reference): `JavaHashMap` below restates
its published algorithm literally — table allocated at the first put with 16
bins, hash(key) = h ^ (h >>> 16) with Short.hashCode(v) = v, new keys appended
to their bin, a bin reaching 9 nodes resized instead of treeified while the
table is under 64 bins, resize doubling when size exceeds 3/4 of the bins with
each bin split in order, remove unlinking.  Pinned by the reference's
SerializationSpec.scala (DeltaShadow 25 / 13 bytes, a two-actor graph of size
2); the HashMap order itself has no fixture in the reference ("parity
unpinned" beyond this restatement of OpenJDK's algorithm).
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

import numpy as np

DELTA_INTERNED, DELTA_ROOT, DELTA_BUSY = 1, 2, 4
ENTRY_BUSY, ENTRY_ROOT = 1, 2
NO_ACTOR = (1 << 64) - 1


def _i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


class JavaHashMap:
    """java.util.HashMap restated for put / get / remove / iteration."""

    TREEIFY_THRESHOLD, MIN_TREEIFY_CAPACITY = 8, 64

    def __init__(self):
        self.table = None  # list of bins, each a list of [key, value] in list order
        self.size = 0
        self.threshold = 0

    @staticmethod
    def _hash(key: int) -> int:
        h = key & 0xFFFFFFFF  # Short.hashCode: the value, as an int
        return (h ^ (h >> 16)) & 0xFFFFFFFF

    def _resize(self):
        old = self.table
        cap = 16 if old is None else 2 * len(old)
        new = [[] for _ in range(cap)]
        for b in old or []:
            for node in b:  # lo / hi split keeps each bin's order
                new[self._hash(node[0]) & (cap - 1)].append(node)
        self.table = new
        self.threshold = cap * 3 // 4

    def get(self, key, default=None):
        if self.table is None:
            return default
        for k, v in self.table[self._hash(key) & (len(self.table) - 1)]:
            if k == key:
                return v
        return default

    def put(self, key, value):
        if self.table is None:
            self._resize()
        b = self.table[self._hash(key) & (len(self.table) - 1)]
        for node in b:
            if node[0] == key:
                node[1] = value
                return
        b.append([key, value])
        if len(b) >= self.TREEIFY_THRESHOLD + 1:  # treeifyBin
            if len(self.table) < self.MIN_TREEIFY_CAPACITY:
                self._resize()
            else:
                raise NotImplementedError("tree bins (unreachable for keys < 64)")
        self.size += 1
        if self.size > self.threshold:
            self._resize()

    def remove(self, key):
        if self.table is None:
            return
        b = self.table[self._hash(key) & (len(self.table) - 1)]
        for i, node in enumerate(b):
            if node[0] == key:
                del b[i]
                self.size -= 1
                return

    def items(self) -> List[Tuple[int, int]]:
        return [(k, v) for b in (self.table or []) for k, v in b]

    def __len__(self):
        return self.size


class DeltaShadow:  # DeltaShadow.java:11-51
    def __init__(self):
        self.outgoing = JavaHashMap()
        self.recvCount = 0
        self.supervisor = -1
        self.interned = False
        self.isRoot = False
        self.isBusy = False

    def serialize(self) -> bytes:  # DeltaShadow.java:57-69 (DataOutput, big-endian)
        out = struct.pack(">ih???i", self.recvCount, self.supervisor, self.interned, self.isRoot,
                          self.isBusy, len(self.outgoing))
        for k, v in self.outgoing.items():
            out += struct.pack(">hi", k, v)
        return out


class DeltaGraph:  # DeltaGraph.java:22-187
    def __init__(self, F: int = 4, DGS: int = 64):
        self.F, self.DGS = F, DGS
        self.table: Dict[int, int] = {}
        self.shadows: List[DeltaShadow] = []
        self.refs: List[int] = []

    @property
    def size(self) -> int:
        return len(self.shadows)

    def encode(self, ref: int) -> int:  # :148-156
        c = self.table.get(ref)
        if c is None:
            c = len(self.shadows)
            self.table[ref] = c
            self.shadows.append(DeltaShadow())
            self.refs.append(ref)
        return c

    @staticmethod
    def _update(m: JavaHashMap, key: int, delta: int):  # :127-136
        c = m.get(key, 0)
        if c + delta == 0:
            m.remove(key)
        else:
            m.put(key, _i32(c + delta))

    def merge_entry(self, b, i: int):  # :73-125, entry i of an EntryBatch
        me = self.encode(int(b.self[i]))
        s = self.shadows[me]
        s.interned = True
        s.recvCount = _i32(s.recvCount + int(b.recv_count[i]))
        s.isBusy = bool(b.flags[i] & ENTRY_BUSY)
        s.isRoot = bool(b.flags[i] & ENTRY_ROOT)
        for k in range(int(b.created_off[i]), int(b.created_off[i + 1])):
            t = self.encode(int(b.created_target[k]))
            o = self.encode(int(b.created_owner[k]))
            self._update(self.shadows[o].outgoing, t, 1)
        for k in range(int(b.spawned_off[i]), int(b.spawned_off[i + 1])):
            self.shadows[self.encode(int(b.spawned[k]))].supervisor = me
        for k in range(int(b.updated_off[i]), int(b.updated_off[i + 1])):
            t = self.encode(int(b.updated_ref[k]))
            info = int(b.updated_info[k])
            cnt = info >> 1  # RefobInfo.count: (short)(info >> 1), info a signed short
            if cnt > 0:
                self.shadows[t].recvCount = _i32(self.shadows[t].recvCount - cnt)
            if info & 1:  # !RefobInfo.isActive
                self._update(s.outgoing, t, -1)

    def is_full(self) -> bool:  # :174-180
        return self.size + 4 * self.F + 1 >= self.DGS

    def shadows_bytes(self) -> bytes:  # :196-200
        return struct.pack(">h", self.size) + b"".join(s.serialize() for s in self.shadows)

    def rows(self):
        """Decoded rows (DeltaGraph.decoder, :162-169), outgoing in iteration order."""
        for c, s in enumerate(self.shadows):
            fl = (DELTA_INTERNED if s.interned else 0) | (DELTA_ROOT if s.isRoot else 0) | \
                 (DELTA_BUSY if s.isBusy else 0)
            sup = self.refs[s.supervisor] if s.supervisor >= 0 else NO_ACTOR
            yield (self.refs[c], s.recvCount, sup, fl,
                   [(self.refs[k], v) for k, v in s.outgoing.items()])


def build(batch, F: int = 4, DGS: int = 64) -> List[DeltaGraph]:
    """The wakeup's DeltaGraphs (LocalGC.scala:159-177)."""
    graphs, g = [], DeltaGraph(F, DGS)
    for i in range(batch.n_entries):
        g.merge_entry(batch, i)
        if g.is_full():
            graphs.append(g)
            g = DeltaGraph(F, DGS)
    if g.size:
        graphs.append(g)
    return graphs


def arrays(graphs: List[DeltaGraph]):
    """What crgc_build_delta_graphs returns: decoded columns, graph_off, wire, wire_off."""
    rows = [r for g in graphs for r in g.rows()]
    cols = dict(
        id=np.array([r[0] for r in rows], np.uint64),
        recv_count=np.array([r[1] for r in rows], np.int32),
        supervisor=np.array([r[2] for r in rows], np.uint64),
        flags=np.array([r[3] for r in rows], np.uint8),
        out_off=np.concatenate([[0], np.cumsum([len(r[4]) for r in rows])]).astype(np.uint32),
        out_target=np.array([t for r in rows for t, _ in r[4]], np.uint64),
        out_count=np.array([c for r in rows for _, c in r[4]], np.int32))
    graph_off = np.concatenate([[0], np.cumsum([g.size for g in graphs])]).astype(np.uint32)
    blobs = [g.shadows_bytes() for g in graphs]
    wire = np.frombuffer(b"".join(blobs), np.uint8)
    wire_off = np.concatenate([[0], np.cumsum([len(x) for x in blobs])]).astype(np.uint64)
    return cols, graph_off, wire, wire_off
