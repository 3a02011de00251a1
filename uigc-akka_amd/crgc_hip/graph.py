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
    @staticmethod
    def _result(out, g, k) -> TraceResult:
        st = out.stats
        return TraceResult(g, k, int(out.n_live), int(st.pseudo_roots), int(st.edges_scanned),
                           int(st.sup_edges), int(st.levels), int(st.launches), st.ms_mark,
                           st.ms_sweep, st.ms_total)

    def _trace_into(self, shouldKill, g, k):
        out = abi.CrgcTraceOut()
        out.garbage_ids, out.garbage_cap = _ptr(g), len(g)
        out.kill_ids, out.kill_cap = _ptr(k), len(k)
        rc = self.lib.crgc_trace(self.h, int(bool(shouldKill)), C.byref(out))
        return rc, out

    def trace(self, shouldKill: bool = True) -> TraceResult:
        """ShadowGraph.trace(shouldKill): returns the garbage and kill id sets."""
        r, ng, nk = self.trace_kill_ids(shouldKill)
        return TraceResult(r.garbage[:ng].copy(), r.kill[:nk].copy(), *[
            getattr(r, f) for f in ("n_live", "pseudo_roots", "edges_scanned", "sup_edges",
                                    "levels", "launches", "ms_mark", "ms_sweep", "ms_total")])

    def trace_kill_ids(self, shouldKill: bool = True):
        """trace() into reusable host buffers: (result with buffer views, n_garbage, n_kill)."""
        self.flush()
        if getattr(self, "_gbuf", None) is None:
            self._gbuf = np.zeros(1 << 16, np.uint64)
            self._kbuf = np.zeros(1 << 16, np.uint64)
        rc, out = self._trace_into(shouldKill, self._gbuf, self._kbuf)
        if rc == abi.E2BIG:
            if out.n_garbage > len(self._gbuf):
                self._gbuf = np.zeros(int(out.n_garbage) * 2, np.uint64)
            if out.n_kill > len(self._kbuf):
                self._kbuf = np.zeros(int(out.n_kill) * 2, np.uint64)
            out.garbage_ids, out.garbage_cap = _ptr(self._gbuf), len(self._gbuf)
            out.kill_ids, out.kill_cap = _ptr(self._kbuf), len(self._kbuf)
            rc = self.lib.crgc_last_trace(self.h, C.byref(out))
        self._chk(rc, "crgc_trace")
        ng, nk = int(out.n_garbage), int(out.n_kill)
        return self._result(out, self._gbuf[:ng], self._kbuf[:nk]), ng, nk

    def trace_counts(self, shouldKill: bool = True):
        """trace() without copying the id lists back (counts and timings only)."""
        self.flush()
        out = abi.CrgcTraceOut()
        self._chk(self.lib.crgc_trace(self.h, int(bool(shouldKill)), C.byref(out)), "crgc_trace")
        e = np.zeros(0, np.uint64)
        return self._result(out, e, e), int(out.n_garbage), int(out.n_kill)

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

    def export(self):
        self.flush()
        return export_to_state(self.lib.crgc_export, self.h)
