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
import dataclasses
import sys
from typing import List, Optional

import numpy as np

from . import abi
from .batch import (Entry, EntryBatch, DeltaBatch, UndoBatch, TraceResult, GraphState, _ptr,
                    export_to_state)


def _host_ids(n: int) -> np.ndarray:
    """A host id buffer for trace results: page-locked when the process already
    uses torch (the device copies into it directly), else ordinary memory.
    torch is never imported from here: importing it after this library has
    initialised the HIP runtime makes the process abort in its exit handlers
    (torch's pinned-memory pool outlives the runtime), so a torch-free caller
    stays torch-free."""
    torch = sys.modules.get("torch")
    if torch is not None:
        try:
            if torch.cuda.is_available():
                return torch.empty(n, dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
        except Exception:
            pass
    return np.zeros(n, np.uint64)


class ShadowGraph:
    def __init__(self, entry_field_size: int = 4, delta_graph_size: int = 64,
                 device: int = 0, vertex_capacity: int = 0, edge_capacity: int = 0,
                 stream: Optional[int] = None, n_shards: int = 1, shard: int = 0,
                 transport=None, proxy_capacity: int = 0):
        """One shadow graph, or (n_shards > 1) shard `shard` of a hash-partitioned
        one whose shards exchange through `transport` (a Transport).  Merges,
        traces and investigateRemotelyHeldActors are then collective."""
        self.lib = abi.load_library()
        cfg = abi.CrgcConfig()
        cfg.abi_version = abi.ABI_VERSION
        cfg.device = device
        cfg.entry_field_size = entry_field_size
        cfg.delta_graph_size = delta_graph_size
        cfg.vertex_capacity = vertex_capacity
        cfg.edge_capacity = edge_capacity
        cfg.stream = stream or None
        cfg.n_shards = n_shards
        cfg.shard = shard
        cfg.transport = transport.t if transport is not None else None
        cfg.proxy_capacity = proxy_capacity
        self.n_shards, self.shard = n_shards, shard
        self._transport = transport  # keeps it alive at least as long as this handle
        h = C.c_void_p()
        self._chk(self.lib.crgc_create(C.byref(cfg), C.byref(h)), "crgc_create")
        self.h = h
        self.F = entry_field_size
        self.DGS = delta_graph_size
        self.device = device
        self._pending: List[Entry] = []
        # Device batches (torch tensors) whose merges may still be running on
        # the graph's stream: held until the next call that synchronises it, so
        # the caching allocator cannot hand their memory to a later copy.
        self._inflight: list = []

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
            raise abi.CrgcError(rc, where, abi.last_error_detail())

    # -- merges ---------------------------------------------------------------
    def mergeEntry(self, entry: Entry):
        """Queue one entry; it is merged (in order) at the next trace/flush."""
        self._pending.append(entry)

    def flush(self):
        if self._pending:
            b = EntryBatch.from_entries(self._pending)
            self._pending = []
            self.merge_entries(b)

    def _hold(self, batch):
        if batch.memory == abi.MEM_DEVICE:
            self._inflight.append(batch)

    def _synced(self):
        """The graph's stream has drained: device batches may be freed."""
        self._inflight.clear()

    def merge_entries(self, batch: EntryBatch):
        self._chk(self.lib.crgc_merge_entries(self.h, C.byref(batch.struct())),
                  "crgc_merge_entries")
        self._hold(batch)

    def merge_entries_async(self, batch: EntryBatch):
        """crgc_merge_entries_async: a batch packed into registered host memory
        is only enqueued (its buffers must stay unchanged until the next trace or
        sync); any other batch merges as merge_entries does."""
        self._chk(self.lib.crgc_merge_entries_async(self.h, C.byref(batch.struct())),
                  "crgc_merge_entries_async")
        self._hold(batch)
        if batch.memory == abi.MEM_HOST:
            self._inflight.append(batch)  # (its arrays stay referenced until the stream drains)

    def merge_deltas(self, batch: DeltaBatch):
        self.flush()
        self._chk(self.lib.crgc_merge_deltas(self.h, C.byref(batch.struct())),
                  "crgc_merge_deltas")
        self._hold(batch)

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
                           st.ms_sweep, st.ms_total, st.ms_frontier, st.ms_tail, st.ms_expand,
                           int(st.rounds), int(st.ids_sent), st.ms_exchange,
                           int(st.expand_launches), int(st.expand_bytes), int(st.exchange_bytes),
                           int(st.time_query_failures), int(st.direct_lists))

    def _trace_into(self, shouldKill, g, k):
        out = abi.CrgcTraceOut()
        out.garbage_ids, out.garbage_cap = _ptr(g), len(g)
        out.kill_ids, out.kill_cap = _ptr(k), len(k)
        rc = self.lib.crgc_trace(self.h, int(bool(shouldKill)), C.byref(out))
        return rc, out

    def trace(self, shouldKill: bool = True) -> TraceResult:
        """ShadowGraph.trace(shouldKill): returns the garbage and kill id sets."""
        r, ng, nk = self.trace_kill_ids(shouldKill)
        return dataclasses.replace(r, garbage=r.garbage[:ng].copy(), kill=r.kill[:nk].copy())

    @staticmethod
    def id_buffers(n: int = 1 << 16):
        """A (garbage, kill) pair of host id buffers for trace_kill_ids(bufs=...):
        page-locked when the process uses torch (the device stores into them)."""
        return _host_ids(n), _host_ids(n)

    def trace_kill_ids(self, shouldKill: bool = True, bufs=None):
        """trace() into reusable host buffers: (result with buffer views, n_garbage, n_kill).
        bufs: the caller's (garbage, kill) buffers (id_buffers()) instead of the
        graph's own, for results that must outlive the next trace (a list that
        does not fit comes back in a fresh buffer instead)."""
        self.flush()
        if bufs is None:
            if getattr(self, "_gbuf", None) is None:
                self._gbuf = _host_ids(1 << 16)
                self._kbuf = _host_ids(1 << 16)
            gb, kb = self._gbuf, self._kbuf
        else:
            gb, kb = bufs
        rc, out = self._trace_into(shouldKill, gb, kb)
        if rc == abi.E2BIG:
            if out.n_garbage > len(gb):
                gb = _host_ids(int(out.n_garbage) * 2)
            if out.n_kill > len(kb):
                kb = _host_ids(int(out.n_kill) * 2)
            if bufs is None:
                self._gbuf, self._kbuf = gb, kb
            out.garbage_ids, out.garbage_cap = _ptr(gb), len(gb)
            out.kill_ids, out.kill_cap = _ptr(kb), len(kb)
            rc = self.lib.crgc_last_trace(self.h, C.byref(out))
        self._synced()
        self._chk(rc, "crgc_trace")
        ng, nk = int(out.n_garbage), int(out.n_kill)
        return self._result(out, gb[:ng], kb[:nk]), ng, nk

    def trace_counts(self, shouldKill: bool = True):
        """trace() without copying the id lists back (counts and timings only)."""
        self.flush()
        out = abi.CrgcTraceOut()
        rc = self.lib.crgc_trace(self.h, int(bool(shouldKill)), C.byref(out))
        self._synced()
        self._chk(rc, "crgc_trace")
        e = np.zeros(0, np.uint64)
        return self._result(out, e, e), int(out.n_garbage), int(out.n_kill)

    def last_trace(self):
        """The retained lists of the last trace (crgc_last_trace), as a fresh
        (garbage, kill) pair of arrays: the second phase of a two-phase trace."""
        out = abi.CrgcTraceOut()
        self._chk(self.lib.crgc_last_trace(self.h, C.byref(out)), "crgc_last_trace")
        g = np.zeros(max(1, int(out.n_garbage)), np.uint64)
        k = np.zeros(max(1, int(out.n_kill)), np.uint64)
        out.garbage_ids, out.garbage_cap = _ptr(g), len(g)
        out.kill_ids, out.kill_cap = _ptr(k), len(k)
        self._chk(self.lib.crgc_last_trace(self.h, C.byref(out)), "crgc_last_trace")
        return g[:int(out.n_garbage)], k[:int(out.n_kill)]

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

    def register_host(self, buf: np.ndarray):
        """Pin a host buffer for DMA (crgc_host_register): batches packed into it
        (HostArena) are copied without the driver's pageable staging."""
        self._chk(self.lib.crgc_host_register(self.h, buf.ctypes.data, buf.nbytes), "crgc_host_register")

    def unregister_host(self, buf: np.ndarray):
        """Unpin `buf` (crgc_host_unregister): pending entries are merged first, and
        the call waits for async merges still reading it."""
        self.flush()
        self._chk(self.lib.crgc_host_unregister(self.h, buf.ctypes.data), "crgc_host_unregister")
        self._synced()

    def usage(self) -> dict:
        """Slot and table usage (crgc_usage_of): slot_top counts the slots of
        collected shadows not yet reused; the dense trace passes scale with it."""
        u = abi.CrgcUsage()
        self._chk(self.lib.crgc_usage_of(self.h, C.byref(u)), "crgc_usage_of")
        return {n: int(getattr(u, n)) for n, _ in abi.CrgcUsage._fields_}

    def compact(self):
        """Compact the graph now (crgc_compact): dense slots, segments in slot order."""
        self.flush()
        self._chk(self.lib.crgc_compact(self.h), "crgc_compact")

    def live_count(self) -> int:
        self.flush()
        v = C.c_uint64()
        self._chk(self.lib.crgc_live_count(self.h, C.byref(v)), "crgc_live_count")
        return v.value

    def export(self):
        self.flush()
        return export_to_state(self.lib.crgc_export, self.h)

    def undo_accumulator(self, node_location: int) -> "UndoAccumulator":
        return UndoAccumulator(self, node_location)

    def merge_undo_acc(self, acc: "UndoAccumulator"):
        """ShadowGraph.mergeUndoLog(undoLogs(address)) with a device-folded log."""
        self.flush()
        self._chk(self.lib.crgc_merge_undo_acc(self.h, acc.h), "crgc_merge_undo_acc")

    # -- DeltaGraph production (num-nodes > 1, LocalGC.scala:159-177) --------------
    def sync(self):
        """Wait for everything queued on the graph's stream (crgc_sync)."""
        self._chk(self.lib.crgc_sync(self.h), "crgc_sync")
        self._synced()

    def build_delta_graphs(self, batch: EntryBatch, device_out: bool = False, sync: bool = True):
        """The wakeup's entries folded into DeltaGraphs on the device
        (DeltaGraph.java:73-180).  Returns (DeltaBatch of the decoded shadows,
        graph_off, wire bytes, wire_off): graph g is shadows
        graph_off[g]:graph_off[g+1] and payload bytes wire[wire_off[g]:wire_off[g+1]]
        (writeShort(size) + DeltaShadow.serialize per shadow).  device_out: the
        arrays are torch tensors on the graph's device.  The returned arrays are
        views of buffers reused by the next call with the same device_out.  Device
        outputs are stream-ordered: sync=False leaves them to work the caller queues
        on the graph's stream."""
        s = batch.struct()
        key = "_dg_dev" if device_out else "_dg_host"
        bufs = getattr(self, key, None)
        q = abi.CrgcDeltaGraphs()
        for attempt in range(2):
            q.memory = abi.MEM_DEVICE if device_out else abi.MEM_HOST
            if bufs is not None:
                arrs, caps = bufs
                for k, v in arrs.items():
                    setattr(q, k, _ptr(v))
                q.graph_cap, q.shadow_cap, q.out_cap, q.wire_cap = caps
            rc = self.lib.crgc_build_delta_graphs(self.h, C.byref(s), C.byref(q))
            if rc == abi.OK and bufs is not None:
                break
            if rc not in (abi.OK, abi.E2BIG):
                self._chk(rc, "crgc_build_delta_graphs")
            caps = tuple(int(x * 1.25) + 16 for x in (q.n_graphs, q.n_shadows, q.n_out, q.wire_bytes))
            bufs = (self._dg_buffers(device_out, *caps), caps)
            setattr(self, key, bufs)
        else:
            self._chk(rc, "crgc_build_delta_graphs")
        if device_out and sync:
            self.sync()
        arrs = bufs[0]
        G, NS, NO, NW = q.n_graphs, q.n_shadows, q.n_out, q.wire_bytes
        cut = lambda k, n: arrs[k][:n]  # noqa: E731
        mem = abi.MEM_DEVICE if device_out else abi.MEM_HOST
        deltas = DeltaBatch(cut("id", NS), cut("recv_count", NS), cut("supervisor", NS),
                            cut("flags", NS), cut("out_off", NS + 1), cut("out_target", NO),
                            cut("out_count", NO), memory=mem)
        return deltas, cut("graph_off", G + 1), cut("wire", NW), cut("wire_off", G + 1)

    def _dg_buffers(self, device_out, G, NS, NO, NW):
        if device_out:
            import torch
            dev = f"cuda:{self.device}"
            mk = lambda n, dt: torch.empty(n, dtype=dt, device=dev)  # noqa: E731
            u8, i32, u32, u64 = torch.uint8, torch.int32, torch.uint32, torch.uint64
        else:
            mk = lambda n, dt: np.zeros(n, dtype=dt)  # noqa: E731
            u8, i32, u32, u64 = np.uint8, np.int32, np.uint32, np.uint64
        return dict(graph_off=mk(G + 1, u32), wire_off=mk(G + 1, u64), id=mk(NS, u64),
                    recv_count=mk(NS, i32), supervisor=mk(NS, u64), flags=mk(NS, u8),
                    out_off=mk(NS + 1, u32), out_target=mk(NO, u64), out_count=mk(NO, i32),
                    wire=mk(NW, u8))


class UndoAccumulator:
    """UndoLog(nodeAddress) kept on the graph's device (UndoLog.java:16-104):
    fold_deltas = mergeDeltaGraph (:39-67, called per DeltaMsg, LocalGC.scala:133),
    fold_ingress = mergeIngressEntry (:69-93); graph.merge_undo_acc(acc) =
    ShadowGraph.mergeUndoLog with it (:158-174).  Close before the graph."""

    def __init__(self, graph: "ShadowGraph", node_location: int):
        self.lib, self.graph = graph.lib, graph
        self.location = node_location
        h = C.c_void_p()
        ShadowGraph._chk(self.lib.crgc_undo_acc_create(graph.h, node_location, C.byref(h)),
                         "crgc_undo_acc_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.crgc_undo_acc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fold_deltas(self, batch: DeltaBatch):
        ShadowGraph._chk(self.lib.crgc_undo_acc_fold_deltas(self.h, C.byref(batch.struct())),
                         "crgc_undo_acc_fold_deltas")
        self.graph._hold(batch)

    mergeDeltaGraph = fold_deltas

    def fold_ingress(self, fields: UndoBatch):
        ShadowGraph._chk(self.lib.crgc_undo_acc_fold_ingress(self.h, C.byref(fields.struct())),
                         "crgc_undo_acc_fold_ingress")
        self.graph._hold(fields)  # device input: read on the stream after the call returns

    mergeIngressEntry = fold_ingress

    def export(self) -> UndoBatch:
        q = abi.CrgcUndoLogOut()
        ShadowGraph._chk(self.lib.crgc_undo_acc_export(self.h, C.byref(q)), "crgc_undo_acc_export")
        nf, nc = int(q.n_fields), int(q.n_created)
        actor, msg = np.zeros(nf + 1, np.uint64), np.zeros(nf + 1, np.int32)
        off = np.zeros(nf + 1, np.uint32)
        tgt, cnt = np.zeros(nc + 1, np.uint64), np.zeros(nc + 1, np.int32)
        q.actor, q.message_count, q.created_off = _ptr(actor), _ptr(msg), _ptr(off)
        q.created_target, q.created_count = _ptr(tgt), _ptr(cnt)
        q.field_cap, q.created_cap = nf, nc
        ShadowGraph._chk(self.lib.crgc_undo_acc_export(self.h, C.byref(q)), "crgc_undo_acc_export")
        return UndoBatch(self.location, actor[:nf], msg[:nf], off, tgt[:nc], cnt[:nc])


class Transport:
    """A shard transport (include/crgc.h): RCCL over xGMI between processes, or
    in-process device copies between G shards driven by G host threads."""

    def __init__(self, handle, lib):
        self.t, self.lib = handle, lib

    @classmethod
    def local(cls, n_shards: int) -> "Transport":
        lib = abi.load_library()
        t = C.c_void_p()
        ShadowGraph._chk(lib.crgc_transport_local(n_shards, C.byref(t)), "crgc_transport_local")
        return cls(t, lib)

    @staticmethod
    def rccl_unique_id() -> bytes:
        lib = abi.load_library()
        buf = C.create_string_buffer(128)
        ShadowGraph._chk(lib.crgc_transport_rccl_id(buf), "crgc_transport_rccl_id")
        return buf.raw

    @classmethod
    def rccl(cls, uid: bytes, n_shards: int, shard: int, device: int) -> "Transport":
        lib = abi.load_library()
        t = C.c_void_p()
        ShadowGraph._chk(lib.crgc_transport_rccl(uid, n_shards, shard, device, C.byref(t)),
                         "crgc_transport_rccl")
        return cls(t, lib)

    @classmethod
    def host(cls, collectives: "HostCollectives", device: int) -> "Transport":
        """crgc_transport_host: this process's shard over host collectives
        (`collectives`, e.g. GlooCollectives: torch.distributed over gloo)."""
        lib = abi.load_library()
        t = C.c_void_p()
        ShadowGraph._chk(lib.crgc_transport_host(C.byref(collectives.c), collectives.n_shards,
                                                 collectives.shard, device, C.byref(t)), "crgc_transport_host")
        tr = cls(t, lib)
        tr._keep = collectives  # the callbacks must outlive the transport
        return tr

    def close(self):
        if self.t:
            self.lib.crgc_transport_destroy(self.t)
            self.t = None


class HostCollectives:
    """The callbacks of crgc_transport_host over torch.distributed (any
    backend with all_gather_into_tensor / all_to_all_single on CPU tensors:
    gloo).  Buffers are the transport's pinned host staging; the callbacks run
    on the thread that called into the graph."""

    def __init__(self, n_shards: int, shard: int, group=None):
        import numpy as np
        import torch
        import torch.distributed as dist
        self.n_shards, self.shard, self.group = n_shards, shard, group
        np_, torch_, dist_ = np, torch, dist

        def view(addr, n):
            return np_.ctypeslib.as_array((C.c_uint8 * max(int(n), 1)).from_address(addr))[:int(n)]

        def allgather(_ctx, _shard, send, recv, nbytes):
            try:
                src = torch_.from_numpy(view(send, nbytes).copy())
                out = torch_.empty(int(nbytes) * n_shards, dtype=torch_.uint8)
                dist_.all_gather_into_tensor(out, src, group=self.group)
                view(recv, int(nbytes) * n_shards)[:] = out.numpy()
                return 0
            except Exception:  # noqa: BLE001 — a failed exchange fails the call, not the process
                return 1

        def alltoallv(_ctx, _shard, send, soff, sbytes, recv, roff, rbytes):
            try:
                sb = [int(sbytes[r]) for r in range(n_shards)]
                rb = [int(rbytes[r]) for r in range(n_shards)]
                sn = max([int(soff[r]) + sb[r] for r in range(n_shards) if sb[r]] or [0])
                rn = max([int(roff[r]) + rb[r] for r in range(n_shards) if rb[r]] or [0])
                sv = view(send, sn)
                inp = torch_.from_numpy(np_.concatenate(
                    [sv[int(soff[r]):int(soff[r]) + sb[r]] for r in range(n_shards)] or [np_.zeros(0, np_.uint8)]))
                out = torch_.empty(sum(rb), dtype=torch_.uint8)
                dist_.all_to_all_single(out, inp, rb, sb, group=self.group)
                rv, o, at = view(recv, rn), out.numpy(), 0
                for r in range(n_shards):
                    rv[int(roff[r]):int(roff[r]) + rb[r]] = o[at:at + rb[r]]
                    at += rb[r]
                return 0
            except Exception:  # noqa: BLE001
                return 1

        self._ag = abi.HOST_ALLGATHER(allgather)
        self._a2a = abi.HOST_ALLTOALLV(alltoallv)
        self.c = abi.HostCollectives(None, self._ag, self._a2a)


def shard_of(actor_id: int, n_shards: int) -> int:
    """Home shard of an actor id (crgc_shard_of)."""
    return int(abi.load_library().crgc_shard_of(actor_id, n_shards))


class ShardedShadowGraph:
    """G shards of one hash-partitioned shadow graph in this process, each on
    its own host thread (collective calls run on all shards at once) over the
    in-process transport.  `devices` may repeat a GPU: G logical shards on one
    MI355X run exactly the protocol of G shards on G GPUs, with device copies
    in place of RCCL.  Results are the union over shards (garbage, kill) or
    sums (counts), which is what one unsharded ShadowGraph returns.
    """

    def __init__(self, n_shards: int, devices=None, entry_field_size: int = 4,
                 vertex_capacity: int = 0, edge_capacity: int = 0, proxy_capacity: int = 0,
                 stream: Optional[int] = None):
        """stream: one hipStream_t for every shard (a diagnostic: the shards'
        kernels then run one at a time, so a kernel trace shows each one's own
        duration); default, each shard its own stream."""
        import concurrent.futures as cf
        self.G = n_shards
        devices = list(devices) if devices is not None else [0] * n_shards
        self.transport = Transport.local(n_shards)
        self.shards = [ShadowGraph(entry_field_size=entry_field_size, device=devices[r],
                                   vertex_capacity=vertex_capacity, edge_capacity=edge_capacity,
                                   n_shards=n_shards, shard=r, transport=self.transport,
                                   proxy_capacity=proxy_capacity, stream=stream)
                       for r in range(n_shards)]
        self._pool = cf.ThreadPoolExecutor(max_workers=n_shards)

    def _all(self, fn, args=None):
        args = args if args is not None else [()] * self.G
        futs = [self._pool.submit(fn, s, *a) for s, a in zip(self.shards, args)]
        return [f.result() for f in futs]

    def close(self):
        for s in self.shards:
            s.close()
        self.transport.close()
        self._pool.shutdown()

    # -- collective -------------------------------------------------------------
    def merge_entries(self, batch, split: bool = False):
        """Merge one batch.  By default shard 0 contributes it and the others
        contribute nothing; with split=True it is cut into G consecutive parts,
        shard r contributing part r (the merge applies them in shard order, so
        the result is the same)."""
        parts = batch.split(self.G) if split else [batch] + [None] * (self.G - 1)
        self._all(lambda s, b: s.merge_entries(b if b is not None else EntryBatch.empty()),
                  [(p,) for p in parts])

    def merge_parts(self, parts):
        """Merge one batch given as G per-shard parts (host or device batches; part r
        contributed by shard r), applied in shard order."""
        assert len(parts) == self.G
        self._all(lambda s, b: s.merge_entries(b if b is not None else EntryBatch.empty()),
                  [(p,) for p in parts])

    def merge_deltas(self, batch):
        self._all(lambda s, b: s.merge_deltas(b if b is not None else DeltaBatch.empty()),
                  [(batch,)] + [(None,)] * (self.G - 1))

    def merge_undo(self, log):
        self._all(lambda s: s.merge_undo(log))

    def trace(self, shouldKill: bool = True) -> TraceResult:
        rs = self._all(lambda s: s.trace(shouldKill))
        return TraceResult(
            np.concatenate([r.garbage for r in rs]), np.concatenate([r.kill for r in rs]),
            sum(r.n_live for r in rs), sum(r.pseudo_roots for r in rs),
            sum(r.edges_scanned for r in rs), sum(r.sup_edges for r in rs),
            max(r.levels for r in rs), sum(r.launches for r in rs),
            max(r.ms_mark for r in rs), max(r.ms_sweep for r in rs), max(r.ms_total for r in rs),
            max(r.ms_frontier for r in rs), max(r.ms_tail for r in rs),
            max(r.ms_expand for r in rs), max(r.rounds for r in rs),
            sum(r.ids_sent for r in rs), max(r.ms_exchange for r in rs),
            sum(r.expand_launches for r in rs), sum(r.expand_bytes for r in rs),
            sum(r.exchange_bytes for r in rs), sum(r.time_query_failures for r in rs),
            min(r.direct_lists for r in rs))

    def count_reachable_from(self, location: int) -> int:
        vals = self._all(lambda s: s.count_reachable_from(location))
        assert len(set(vals)) == 1, vals
        return vals[0]

    # -- per shard ------------------------------------------------------------
    def total_actors_seen(self) -> int:
        return sum(s.total_actors_seen() for s in self.shards)

    def live_count(self) -> int:
        return sum(s.live_count() for s in self.shards)

    def compact(self):
        self._all(lambda s: s.compact())

    def startWave(self):
        return np.concatenate([s.startWave() for s in self.shards])

    def export(self):
        parts = [s.export() for s in self.shards]
        verts, edges = {}, {}
        for p in parts:
            assert not (verts.keys() & p.vertices.keys()), "a shadow on two shards"
            verts.update(p.vertices)
            assert not (edges.keys() & p.edges.keys()), "an edge on two shards"
            edges.update(p.edges)
        return GraphState(verts, edges)
