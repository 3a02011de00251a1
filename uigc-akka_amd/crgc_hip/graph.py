"""`ShadowGraph` — the reference's collector-side surface over the HIP shim.

Method names follow the reference's ShadowGraph (ShadowGraph.java) so that a
caller written against it reads the same:

    reference (Java)                          here
    new ShadowGraph(context)         :17      ShadowGraph(entry_field_size=4, ...)
    mergeEntry(entry)                :75      mergeEntry(entry)   (buffered) /
                                              merge_entries(EntryBatch)
    mergeDelta(delta)               :127      merge_deltas(DeltaBatch)
    mergeUndoLog(log)               :158      merge_undo(UndoBatch)
    trace(shouldKill)               :205      trace(shouldKill) -> TraceResult
    startWave()                     :291      startWave() -> ids to tell WaveMsg
    investigateRemotelyHeldActors() :302      investigateRemotelyHeldActors(loc)
    totalActorsSeen                  :12      totalActorsSeen

Errors come back as CrgcError with the C code; where the reference throws
(NPE at :277, CME at :162) the codes are E_NULL_SUPERVISOR / E_UNDO_NEW_SHADOW.
There is no CPU fallback: without the built library this raises.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional

import numpy as np

from . import abi
from .batch import (Entry, EntryBatch, DeltaBatch, UndoBatch, TraceResult, _ptr,
                    export_to_state)


class ShadowGraph:
    def __init__(self, entry_field_size: int = 4, delta_graph_size: int = 64,
                 device: int = 0, vertex_capacity: int = 0, edge_capacity: int = 0,
                 stream: Optional[int] = None):
        self.lib = abi.load_library()
        cfg = abi.CrgcConfig()
        cfg.abi_version = abi.ABI_VERSION
        cfg.device = device
        cfg.entry_field_size = entry_field_size
        cfg.delta_graph_size = delta_graph_size
        cfg.vertex_capacity = vertex_capacity
        cfg.edge_capacity = edge_capacity
        cfg.stream = stream or None
        h = C.c_void_p()
        self._chk(self.lib.crgc_create(C.byref(cfg), C.byref(h)), "crgc_create")
        self.h = h
        self.F = entry_field_size
        self._pending: List[Entry] = []

    # -- lifecycle ------------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.crgc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @staticmethod
    def _chk(rc: int, where: str):
        if rc != abi.OK:
            raise abi.CrgcError(rc, where)

    # -- merges ---------------------------------------------------------------
    def mergeEntry(self, entry: Entry):
        """Queue one entry; it is merged (in order) at the next trace/flush."""
        self._pending.append(entry)

    def flush(self):
        if self._pending:
            b = EntryBatch.from_entries(self._pending)
            self._pending = []
            self.merge_entries(b)

    def merge_entries(self, batch: EntryBatch):
        self._chk(self.lib.crgc_merge_entries(self.h, C.byref(batch.struct())),
                  "crgc_merge_entries")

    def merge_deltas(self, batch: DeltaBatch):
        self.flush()
        self._chk(self.lib.crgc_merge_deltas(self.h, C.byref(batch.struct())),
                  "crgc_merge_deltas")

    def merge_undo(self, log: UndoBatch):
        self.flush()
        self._chk(self.lib.crgc_merge_undo(self.h, C.byref(log.struct())), "crgc_merge_undo")

    mergeDelta = merge_deltas
    mergeUndoLog = merge_undo

    # -- trace ----------------------------------------------------------------
    def trace(self, shouldKill: bool = True, capacity: Optional[int] = None) -> TraceResult:
        self.flush()
        cap = capacity if capacity is not None else self.live_count_upper()
        g = np.zeros(max(cap, 1), np.uint64)
        k = np.zeros(max(cap, 1), np.uint64)
        out = abi.CrgcTraceOut()
        out.garbage_ids, out.garbage_cap = _ptr(g), cap
        out.kill_ids, out.kill_cap = _ptr(k), cap
        rc = self.lib.crgc_trace(self.h, int(bool(shouldKill)), C.byref(out))
        if rc == abi.E2BIG:
            g = np.zeros(max(int(out.n_garbage), 1), np.uint64)
            k = np.zeros(max(int(out.n_kill), 1), np.uint64)
            out.garbage_ids, out.garbage_cap = _ptr(g), int(out.n_garbage)
            out.kill_ids, out.kill_cap = _ptr(k), int(out.n_kill)
            rc = self.lib.crgc_last_trace(self.h, C.byref(out))
        self._chk(rc, "crgc_trace")
        st = out.stats
        return TraceResult(g[:out.n_garbage].copy(), k[:out.n_kill].copy(), int(out.n_live),
                           int(st.pseudo_roots), int(st.edges_scanned), int(st.sup_edges),
                           int(st.levels), st.ms_mark, st.ms_sweep, st.ms_total)

    def trace_counts(self, shouldKill: bool = True) -> TraceResult:
        """trace() without copying the id lists back (counts and timings only)."""
        self.flush()
        out = abi.CrgcTraceOut()
        self._chk(self.lib.crgc_trace(self.h, int(bool(shouldKill)), C.byref(out)), "crgc_trace")
        st = out.stats
        e = np.zeros(0, np.uint64)
        return TraceResult(e, e, int(out.n_live), int(st.pseudo_roots), int(st.edges_scanned),
                           int(st.sup_edges), int(st.levels), st.ms_mark, st.ms_sweep,
                           st.ms_total), int(out.n_garbage), int(out.n_kill)

    # -- queries --------------------------------------------------------------
    def startWave(self) -> np.ndarray:
        self.flush()
        n = C.c_uint64()
        self._chk(self.lib.crgc_local_roots(self.h, None, 0, C.byref(n)), "crgc_local_roots")
        buf = np.zeros(max(n.value, 1), np.uint64)
        self._chk(self.lib.crgc_local_roots(self.h, _ptr(buf), n.value, C.byref(n)),
                  "crgc_local_roots")
        return buf[:n.value].copy()

    local_roots = startWave

    def investigateRemotelyHeldActors(self, location: int) -> int:
        self.flush()
        v = C.c_int64()
        self._chk(self.lib.crgc_count_reachable_from(self.h, location, C.byref(v)),
                  "crgc_count_reachable_from")
        return v.value

    count_reachable_from = investigateRemotelyHeldActors

    @property
    def totalActorsSeen(self) -> int:
        self.flush()
        v = C.c_uint64()
        self._chk(self.lib.crgc_total_actors_seen(self.h, C.byref(v)), "crgc_total_actors_seen")
        return v.value

    def total_actors_seen(self) -> int:
        return self.totalActorsSeen

    def live_count(self) -> int:
        self.flush()
        v = C.c_uint64()
        self._chk(self.lib.crgc_live_count(self.h, C.byref(v)), "crgc_live_count")
        return v.value

    def live_count_upper(self) -> int:
        return self.totalActorsSeen  # every live shadow was created at some point

    def export(self):
        self.flush()
        return export_to_state(self.lib.crgc_export, self.h)
