"""Packed struct-of-arrays batches handed across the C ABI.

`Entry` mirrors the reference's Entry record (Entry.java:5-37).  An
`EntryBatch` is the wire form LocalGC's Wakeup handler would build from the
entries it polls (LocalGC.scala:152-172): one row per entry in queue order,
flat created/spawned/updated arrays with per-entry offsets (the reference's
null-terminated prefixes, ShadowGraph.java:86,97,108).

Batches live in host numpy arrays; `to_device()` copies them into HBM as torch
tensors so a timed region can start with inputs already resident.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Iterable, List, Sequence, Tuple

import numpy as np

from . import abi


def _ptr(a) -> int:
    """Data pointer of a numpy array or torch tensor (0 for empty)."""
    if a is None:
        return 0
    if isinstance(a, np.ndarray):
        return a.ctypes.data if a.size else 0
    return a.data_ptr() if a.numel() else 0


def _offsets(counts: Sequence[int]) -> np.ndarray:
    off = np.zeros(len(counts) + 1, dtype=np.uint32)
    if len(counts):
        off[1:] = np.cumsum(np.asarray(counts, dtype=np.uint64)).astype(np.uint32)
    return off


# --------------------------------------------------------------------------
# RefobInfo (RefobInfo.java:8-35): a 16-bit word, count = info >> 1,
# deactivated iff the low bit is set.
# --------------------------------------------------------------------------
class RefobInfo:
    activeRefob = 0

    @staticmethod
    def _s16(x: int) -> int:
        x &= 0xFFFF
        return x - 0x10000 if x & 0x8000 else x

    @staticmethod
    def canIncrement(info: int) -> bool:
        return info <= 32767 - 2

    @staticmethod
    def incSendCount(info: int) -> int:
        return RefobInfo._s16(info + 2)

    @staticmethod
    def resetCount(info: int) -> int:
        return 0

    @staticmethod
    def count(info: int) -> int:
        return RefobInfo._s16(RefobInfo._s16(info) >> 1)

    @staticmethod
    def isActive(info: int) -> bool:
        return (info & 1) == 0

    @staticmethod
    def deactivate(info: int) -> int:
        return RefobInfo._s16(info | 1)


@dataclass
class Entry:
    """Entry.java:5-37 with actor ids in place of Refobs."""
    self: int
    createdOwners: List[int] = field(default_factory=list)
    createdTargets: List[int] = field(default_factory=list)
    spawnedActors: List[int] = field(default_factory=list)
    updatedRefs: List[int] = field(default_factory=list)
    updatedInfos: List[int] = field(default_factory=list)
    recvCount: int = 0
    isBusy: bool = False
    isRoot: bool = False


class EntryBatch:
    """Packed SoA batch of entries (crgc_entry_batch)."""

    __slots__ = ("self", "recv_count", "flags", "created_off", "created_owner",
                 "created_target", "spawned_off", "spawned", "updated_off",
                 "updated_ref", "updated_info", "memory", "_struct")

    def __init__(self, self_ids, recv_count, flags, created_off, created_owner,
                 created_target, spawned_off, spawned, updated_off, updated_ref,
                 updated_info, memory=abi.MEM_HOST):
        self.self = self_ids
        self.recv_count = recv_count
        self.flags = flags
        self.created_off = created_off
        self.created_owner = created_owner
        self.created_target = created_target
        self.spawned_off = spawned_off
        self.spawned = spawned
        self.updated_off = updated_off
        self.updated_ref = updated_ref
        self.updated_info = updated_info
        self.memory = memory
        self._struct = None

    # -- construction -------------------------------------------------------
    @staticmethod
    def from_entries(entries: Iterable[Entry]) -> "EntryBatch":
        entries = list(entries)
        n = len(entries)
        self_ids = np.array([e.self for e in entries], dtype=np.uint64)
        recv = np.array([e.recvCount for e in entries], dtype=np.int16)
        flags = np.array([(abi.ENTRY_BUSY if e.isBusy else 0) |
                          (abi.ENTRY_ROOT if e.isRoot else 0) for e in entries],
                         dtype=np.uint8)
        c_off = _offsets([len(e.createdOwners) for e in entries])
        s_off = _offsets([len(e.spawnedActors) for e in entries])
        u_off = _offsets([len(e.updatedRefs) for e in entries])
        c_own = np.array([x for e in entries for x in e.createdOwners], dtype=np.uint64)
        c_tgt = np.array([x for e in entries for x in e.createdTargets], dtype=np.uint64)
        sp = np.array([x for e in entries for x in e.spawnedActors], dtype=np.uint64)
        u_ref = np.array([x for e in entries for x in e.updatedRefs], dtype=np.uint64)
        u_inf = np.array([RefobInfo._s16(x) for e in entries for x in e.updatedInfos],
                         dtype=np.int16)
        assert len(self_ids) == n
        return EntryBatch(self_ids, recv, flags, c_off, c_own, c_tgt, s_off, sp,
                          u_off, u_ref, u_inf)

    @staticmethod
    def empty() -> "EntryBatch":
        return EntryBatch.from_entries([])

    @property
    def n_entries(self) -> int:
        return int(self.self.shape[0])

    def n_records(self) -> Tuple[int, int, int]:
        return (int(self.created_owner.shape[0]), int(self.spawned.shape[0]),
                int(self.updated_ref.shape[0]))

    def nbytes(self) -> int:
        tot = 0
        for k in self.__slots__[:11]:
            a = getattr(self, k)
            tot += a.nbytes if isinstance(a, np.ndarray) else a.numel() * a.element_size()
        return tot

    def slice(self, lo: int, hi: int) -> "EntryBatch":
        """Entries [lo, hi) as a new host batch (offsets rebased)."""
        assert self.memory == abi.MEM_HOST
        co, so, uo = self.created_off, self.spawned_off, self.updated_off
        return EntryBatch(
            self.self[lo:hi].copy(), self.recv_count[lo:hi].copy(), self.flags[lo:hi].copy(),
            (co[lo:hi + 1] - co[lo]).astype(np.uint32),
            self.created_owner[co[lo]:co[hi]].copy(), self.created_target[co[lo]:co[hi]].copy(),
            (so[lo:hi + 1] - so[lo]).astype(np.uint32), self.spawned[so[lo]:so[hi]].copy(),
            (uo[lo:hi + 1] - uo[lo]).astype(np.uint32),
            self.updated_ref[uo[lo]:uo[hi]].copy(), self.updated_info[uo[lo]:uo[hi]].copy())

    @staticmethod
    def concat(batches: Sequence["EntryBatch"]) -> "EntryBatch":
        """Host batches back to back, in order (offsets rebased): the queue of
        several producers drained one after the other."""
        bs = [b for b in batches if b.n_entries]
        if not bs:
            return EntryBatch.empty()
        if len(bs) == 1:
            return bs[0]
        assert all(b.memory == abi.MEM_HOST for b in bs)

        def offs(name):
            parts, base = [np.zeros(1, np.uint64)], 0
            for b in bs:
                o = getattr(b, name).astype(np.uint64)
                parts.append(o[1:] + base)
                base += int(o[-1])
            out = np.concatenate(parts)
            assert out[-1] < (1 << 32)
            return out.astype(np.uint32)

        cat = lambda k: np.concatenate([getattr(b, k) for b in bs])  # noqa: E731
        return EntryBatch(cat("self"), cat("recv_count"), cat("flags"), offs("created_off"),
                          cat("created_owner"), cat("created_target"), offs("spawned_off"),
                          cat("spawned"), offs("updated_off"), cat("updated_ref"), cat("updated_info"))

    def split(self, k: int) -> List["EntryBatch"]:
        """k consecutive host parts (part r = entries [n*r/k, n*(r+1)/k))."""
        n = self.n_entries
        b = [n * i // k for i in range(k + 1)]
        return [self.slice(b[i], b[i + 1]) for i in range(k)]

    def to_entries(self) -> List[Entry]:
        assert self.memory == abi.MEM_HOST
        out = []
        co, so, uo = self.created_off, self.spawned_off, self.updated_off
        for i in range(self.n_entries):
            out.append(Entry(
                self=int(self.self[i]),
                createdOwners=[int(x) for x in self.created_owner[co[i]:co[i + 1]]],
                createdTargets=[int(x) for x in self.created_target[co[i]:co[i + 1]]],
                spawnedActors=[int(x) for x in self.spawned[so[i]:so[i + 1]]],
                updatedRefs=[int(x) for x in self.updated_ref[uo[i]:uo[i + 1]]],
                updatedInfos=[int(x) for x in self.updated_info[uo[i]:uo[i + 1]]],
                recvCount=int(self.recv_count[i]),
                isBusy=bool(self.flags[i] & abi.ENTRY_BUSY),
                isRoot=bool(self.flags[i] & abi.ENTRY_ROOT)))
        return out

    def to_device(self, device="cuda") -> "EntryBatch":
        import torch
        conv = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        return EntryBatch(*(conv(getattr(self, k)) for k in self.__slots__[:11]),
                          memory=abi.MEM_DEVICE)

    def struct(self) -> abi.CrgcEntryBatch:
        s = abi.CrgcEntryBatch()
        s.n_entries = self.n_entries
        s.self = _ptr(self.self)
        s.recv_count = _ptr(self.recv_count)
        s.flags = _ptr(self.flags)
        s.created_off = _ptr(self.created_off)
        s.created_owner = _ptr(self.created_owner)
        s.created_target = _ptr(self.created_target)
        s.spawned_off = _ptr(self.spawned_off)
        s.spawned = _ptr(self.spawned)
        s.updated_off = _ptr(self.updated_off)
        s.updated_ref = _ptr(self.updated_ref)
        s.updated_info = _ptr(self.updated_info)
        s.memory = self.memory
        self._struct = s
        return s


class DeltaBatch:
    """Decoded DeltaGraph shadows in arrival order (crgc_delta_batch)."""

    __slots__ = ("id", "recv_count", "supervisor", "flags", "out_off", "out_target",
                 "out_count", "memory", "_struct")

    def __init__(self, ids, recv_count, supervisor, flags, out_off, out_target, out_count,
                 memory=abi.MEM_HOST):
        self.id = ids
        self.recv_count = recv_count
        self.supervisor = supervisor
        self.flags = flags
        self.out_off = out_off
        self.out_target = out_target
        self.out_count = out_count
        self.memory = memory
        self._struct = None

    @property
    def n_shadows(self) -> int:
        return int(self.id.shape[0])

    @staticmethod
    def from_rows(rows) -> "DeltaBatch":
        """rows: iterable of (id, recv, sup_id_or_NO_ACTOR, flags, [(target, count)])."""
        rows = list(rows)
        return DeltaBatch(
            np.array([r[0] for r in rows], dtype=np.uint64),
            np.array([r[1] for r in rows], dtype=np.int32),
            np.array([r[2] for r in rows], dtype=np.uint64),
            np.array([r[3] for r in rows], dtype=np.uint8),
            _offsets([len(r[4]) for r in rows]),
            np.array([t for r in rows for t, _ in r[4]], dtype=np.uint64),
            np.array([c for r in rows for _, c in r[4]], dtype=np.int32))

    @staticmethod
    def empty() -> "DeltaBatch":
        return DeltaBatch.from_rows([])

    @staticmethod
    def concat(batches: Sequence["DeltaBatch"]) -> "DeltaBatch":
        if not batches:
            return DeltaBatch.from_rows([])
        offs, base = [], 0
        for b in batches:
            offs.append(b.out_off[:-1].astype(np.uint64) + base)
            base += int(b.out_off[-1])
        out_off = np.concatenate(offs + [np.array([base], dtype=np.uint64)]).astype(np.uint32)
        cat = lambda k: np.concatenate([getattr(b, k) for b in batches])  # noqa: E731
        return DeltaBatch(cat("id"), cat("recv_count"), cat("supervisor"), cat("flags"),
                          out_off, cat("out_target"), cat("out_count"))

    def to_device(self, device="cuda") -> "DeltaBatch":
        import torch
        conv = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        return DeltaBatch(*(conv(getattr(self, k)) for k in self.__slots__[:7]),
                          memory=abi.MEM_DEVICE)

    def struct(self) -> abi.CrgcDeltaBatch:
        s = abi.CrgcDeltaBatch()
        s.n_shadows = self.n_shadows
        s.id = _ptr(self.id)
        s.recv_count = _ptr(self.recv_count)
        s.supervisor = _ptr(self.supervisor)
        s.flags = _ptr(self.flags)
        s.out_off = _ptr(self.out_off)
        s.out_target = _ptr(self.out_target)
        s.out_count = _ptr(self.out_count)
        s.memory = self.memory
        self._struct = s
        return s


class UndoBatch:
    """An UndoLog flattened for the ABI (crgc_undo_log)."""

    __slots__ = ("node_location", "actor", "message_count", "created_off",
                 "created_target", "created_count", "memory", "_struct")

    def __init__(self, node_location, actor, message_count, created_off, created_target,
                 created_count, memory=abi.MEM_HOST):
        self.node_location = int(node_location)
        self.actor = actor
        self.message_count = message_count
        self.created_off = created_off
        self.created_target = created_target
        self.created_count = created_count
        self.memory = memory
        self._struct = None

    @property
    def n_fields(self) -> int:
        return int(self.actor.shape[0])

    @staticmethod
    def from_fields(node_location: int, fields) -> "UndoBatch":
        """fields: iterable of (actor_id, message_count, [(target, count)])."""
        fields = list(fields)
        return UndoBatch(
            node_location,
            np.array([f[0] for f in fields], dtype=np.uint64),
            np.array([f[1] for f in fields], dtype=np.int32),
            _offsets([len(f[2]) for f in fields]),
            np.array([t for f in fields for t, _ in f[2]], dtype=np.uint64),
            np.array([c for f in fields for _, c in f[2]], dtype=np.int32))

    def struct(self) -> abi.CrgcUndoLog:
        s = abi.CrgcUndoLog()
        s.node_location = self.node_location
        s.n_fields = self.n_fields
        s.actor = _ptr(self.actor)
        s.message_count = _ptr(self.message_count)
        s.created_off = _ptr(self.created_off)
        s.created_target = _ptr(self.created_target)
        s.created_count = _ptr(self.created_count)
        s.memory = self.memory
        self._struct = s
        return s


@dataclass
class TraceResult:
    garbage: np.ndarray
    kill: np.ndarray
    n_live: int
    pseudo_roots: int = 0
    edges_scanned: int = 0
    sup_edges: int = 0
    levels: int = 0
    launches: int = 0
    ms_mark: float = 0.0
    ms_sweep: float = 0.0
    ms_total: float = 0.0
    ms_frontier: float = 0.0
    ms_tail: float = 0.0
    ms_expand: float = 0.0
    rounds: int = 1
    ids_sent: int = 0
    ms_exchange: float = 0.0
    expand_launches: int = 0
    expand_bytes: int = 0
    exchange_bytes: int = 0
    time_query_failures: int = 0
    direct_lists: int = 0

    def garbage_set(self):
        return set(int(x) for x in self.garbage)

    def kill_set(self):
        return set(int(x) for x in self.kill)


@dataclass
class GraphState:
    """Exported graph, canonicalised for comparison."""
    vertices: dict  # id -> (recv, flags, supervisor)
    edges: dict     # (owner, target) -> count

    def __eq__(self, other):
        return self.vertices == other.vertices and self.edges == other.edges


def export_to_state(fn_export, handle) -> GraphState:
    e = abi.CrgcGraphExport()
    rc = fn_export(handle, C.byref(e))
    if rc not in (abi.OK, abi.E2BIG):
        raise abi.CrgcError(rc, "export(size)")
    nv, ne = int(e.n_vertices), int(e.n_edges)
    ids = np.zeros(nv, np.uint64); rc_ = np.zeros(nv, np.int32)
    fl = np.zeros(nv, np.uint8); sup = np.zeros(nv, np.uint64)
    eo = np.zeros(ne, np.uint64); et = np.zeros(ne, np.uint64); ec = np.zeros(ne, np.int32)
    e.vertex_cap, e.edge_cap = nv, ne
    e.id, e.recv_count, e.flags, e.supervisor = _ptr(ids), _ptr(rc_), _ptr(fl), _ptr(sup)
    e.edge_owner, e.edge_target, e.edge_count = _ptr(eo), _ptr(et), _ptr(ec)
    # keep non-null pointers for empty arrays so the callee writes nothing
    dummy = np.zeros(1, np.uint64)
    if nv == 0:
        e.id = e.recv_count = e.flags = e.supervisor = _ptr(dummy)
    if ne == 0:
        e.edge_owner = e.edge_target = e.edge_count = _ptr(dummy)
    rc = fn_export(handle, C.byref(e))
    if rc != abi.OK:
        raise abi.CrgcError(rc, "export")
    verts = {int(ids[i]): (int(rc_[i]), int(fl[i]), int(sup[i])) for i in range(nv)}
    edges = {(int(eo[i]), int(et[i])): int(ec[i]) for i in range(ne)}
    assert len(verts) == nv, "duplicate vertex ids in export"
    assert len(edges) == ne, "duplicate edges in export"
    return GraphState(verts, edges)


class HostArena:
    """A reused host buffer that entry batches are packed into — what a JVM's
    direct ByteBuffers are to the JNI shim: allocated once,
    registered with the graph (crgc_host_register) so merges DMA from it, and
    refilled by every wakeup's drain loop (LocalGC.scala:152-172)."""

    def __init__(self, nbytes: int):
        self.buf = np.empty(int(nbytes) + 4096, dtype=np.uint8)

    def pack(self, b: "EntryBatch", at: int = 0) -> "EntryBatch":
        """Pack `b` into the arena from byte `at` on (the drain loop packs a
        wakeup's chunks one after the other: pack_end() tells where one ended)."""
        assert b.memory == abi.MEM_HOST
        views, off = [], int(at)
        for k in EntryBatch.__slots__[:11]:
            a = np.ascontiguousarray(getattr(b, k))
            off = (off + 255) & ~255
            if off + a.nbytes > self.buf.nbytes:
                raise ValueError("batch larger than the arena")
            v = self.buf[off:off + a.nbytes].view(a.dtype)
            v[...] = a
            views.append(v)
            off += a.nbytes
        self.end = off
        return EntryBatch(*views)
