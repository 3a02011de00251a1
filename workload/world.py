"""ctypes wrapper of world.cpp: seeded synthetic CRGC entry streams (C1-C4)."""

from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "uigc-akka_amd"))
from crgc_hip.batch import EntryBatch  # noqa: E402

LIB = os.path.join(_HERE, "_build", "libcrgc_workload.so")


class WlBatch(C.Structure):
    _fields_ = [("n", C.c_uint64), ("C", C.c_uint64), ("S", C.c_uint64), ("U", C.c_uint64)] + \
        [(k, C.c_void_p) for k in ("self", "recv", "flags", "c_off", "c_owner", "c_target",
                                   "s_off", "spawned", "u_off", "u_ref", "u_info")]


class WlDeltas(C.Structure):
    _fields_ = [("n_graphs", C.c_uint64), ("n_shadows", C.c_uint64), ("n_out", C.c_uint64)] + \
        [(k, C.c_void_p) for k in ("graph_off", "id", "recv", "sup", "flags", "out_off",
                                   "out_target", "out_count")]


def build(force=False) -> str:
    srcs = [os.path.join(_HERE, f) for f in ("world.cpp", "deltas.cpp")]
    if force or not os.path.exists(LIB) or \
            any(os.path.getmtime(LIB) < os.path.getmtime(s) for s in srcs):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", LIB, *srcs])
    return LIB


_lib = None


def _load():
    global _lib
    if _lib is None:
        build()
        lib = C.CDLL(LIB)
        lib.wl_create.restype = C.c_void_p
        lib.wl_create.argtypes = [C.c_uint64, C.c_uint32, C.c_uint16]
        lib.wl_destroy.argtypes = [C.c_void_p]
        lib.wl_set_mix.argtypes = [C.c_void_p] + [C.c_double] * 5
        lib.wl_set_id_space.argtypes = [C.c_void_p, C.c_uint32]
        lib.wl_bulk_graph.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_double,
                                      C.c_uint32, C.c_uint64]
        lib.wl_chain_graph.argtypes = [C.c_void_p] + [C.c_uint32] * 6
        lib.wl_simulate.argtypes = [C.c_void_p, C.c_uint64]
        lib.wl_uniform_graph.argtypes = [C.c_void_p, C.c_uint64, C.c_double, C.c_uint32, C.c_double]
        lib.wl_wakeup.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_double,
                                  C.c_double]
        for f in ("wl_queued", "wl_n_actors", "wl_n_refobs_held", "wl_n_busy", "wl_n_ready"):
            getattr(lib, f).restype = C.c_uint64
            getattr(lib, f).argtypes = [C.c_void_p]
        lib.wl_take.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(WlBatch)]
        lib.wl_compact.argtypes = [C.c_void_p]
        lib.wl_deltas_create.restype = C.c_void_p
        lib.wl_deltas_destroy.argtypes = [C.c_void_p]
        lib.wl_deltas_build.argtypes = [C.c_void_p, C.POINTER(WlBatch), C.c_uint32, C.c_uint32,
                                        C.POINTER(WlDeltas)]
        _lib = lib
    return _lib


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))),
                                 shape=(n,)).copy()


class World:
    """A simulated node: `seed`, entry-field size F, location id."""

    def __init__(self, seed: int, F: int = 4, location: int = 1):
        self.lib = _load()
        self.h = self.lib.wl_create(seed, F, location)

    def close(self):
        if self.h:
            self.lib.wl_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_id_space(self, k: int):
        """Ids from an injective map of (k, actor index): producers with different
        k never share an id (C4's components).  Call before any graph is built."""
        if self.lib.wl_set_id_space(self.h, k) != 0:
            raise ValueError("wl_set_id_space: actors exist already or k > 65535")

    def set_mix(self, send=0.4, share=0.2, release=0.2, spawn=0.1, actions_per_msg=1.5):
        self.lib.wl_set_mix(self.h, send, share, release, spawn, actions_per_msg)

    def bulk_graph(self, n_actors, n_edges, alpha=2.1, n_roots=None, cap=100000):
        n_roots = n_roots if n_roots is not None else max(1, n_actors // 100)
        self.lib.wl_bulk_graph(self.h, n_actors, n_edges, alpha, n_roots, cap)

    def chain_graph(self, n_chains=100, chain_len=10000, n_sup_chains=10, sup_depth=1000,
                    n_rings=100, ring_len=100):
        self.lib.wl_chain_graph(self.h, n_chains, chain_len, n_sup_chains, sup_depth,
                                n_rings, ring_len)

    def simulate(self, n_entries):
        self.lib.wl_simulate(self.h, n_entries)

    def uniform_graph(self, n_actors, mean_acq=8.0, n_roots=None, dead_frac=0.05):
        """C1 shape: spawn tree, Poisson(mean_acq) uniform acquaintances
        with counts 1 / 2 / -1 (90 / 8 / 2 %), dead components holding dead_frac."""
        n_roots = n_roots if n_roots is not None else max(1, n_actors // 100)
        self.lib.wl_uniform_graph(self.h, n_actors, mean_acq, n_roots, dead_frac)

    def n_busy(self) -> int:
        """Actors mid-turn (their last flushed entry says isBusy)."""
        return self.lib.wl_n_busy(self.h)

    def n_ready(self) -> int:
        """Actors with undelivered mail."""
        return self.lib.wl_n_ready(self.h)

    def wakeup(self, n_entries, busy, pending, apm=(1.0, 3.0)) -> EntryBatch:
        """One wakeup's batch of exactly n_entries with turns in flight at the cut:
        about `busy` actors mid-turn (isBusy) and `pending` with undelivered mail
        (wl_wakeup); apm = (lo, hi) actions per received message."""
        need = n_entries - self.queued()
        if need > 0:
            self.lib.wl_wakeup(self.h, need, busy, pending, apm[0], apm[1])
        return self.take(n_entries)

    def queued(self) -> int:
        return self.lib.wl_queued(self.h)

    def n_actors(self) -> int:
        return self.lib.wl_n_actors(self.h)

    def n_refs(self) -> int:
        return self.lib.wl_n_refobs_held(self.h)

    def take(self, max_entries) -> EntryBatch:
        b = WlBatch()
        self.lib.wl_take(self.h, max_entries, C.byref(b))
        n, nc, ns, nu = b.n, b.C, b.S, b.U
        eb = EntryBatch(
            _arr(b.self, n, np.uint64), _arr(b.recv, n, np.int16), _arr(b.flags, n, np.uint8),
            _arr(b.c_off, n + 1, np.uint32), _arr(b.c_owner, nc, np.uint64),
            _arr(b.c_target, nc, np.uint64), _arr(b.s_off, n + 1, np.uint32),
            _arr(b.spawned, ns, np.uint64), _arr(b.u_off, n + 1, np.uint32),
            _arr(b.u_ref, nu, np.uint64), _arr(b.u_info, nu, np.int16))
        self.lib.wl_compact(self.h)
        return eb

    def batches(self, batch_size):
        """Drain the queue in batches of `batch_size` entries."""
        while self.queued():
            yield self.take(batch_size)

    def wakeup_batch(self, n_entries) -> EntryBatch:
        """Simulate until n_entries are queued and take exactly those."""
        need = n_entries - self.queued()
        if need > 0:
            self.simulate(need)
        return self.take(n_entries)


C4_PRODUCERS = 8


def c4_producer(k: int, n_actors: int, n_edges: int) -> World:
    """Producer k (0..7) of BASELINE.json's C4 node: 1/8 of the actors and edges
    of one power-law shadow graph (C2's distribution), location 1,
    id space k + 1 (disjoint from every other producer's).  The union of the 8
    producers' streams is one graph whatever the GPU count that holds it."""
    w = World(seed=0x5EED + 4 + 1000 * k, location=1)
    w.set_id_space(k + 1)
    w.bulk_graph(n_actors, n_edges, alpha=2.1, n_roots=max(1, n_actors // 1000), cap=100000)
    return w


def deltas_of(batch: EntryBatch, F: int = 4, dgs: int = 64):
    """A remote node's drained entries folded into DeltaGraphs
    (LocalGC.scala:159-177 over DeltaGraph.java:73-180; workload/deltas.cpp):
    returns (DeltaBatch of the decoded shadows in graph order, graph offsets)."""
    from crgc_hip.batch import DeltaBatch
    lib = _load()
    wb = WlBatch()
    wb.n = batch.n_entries
    keep = []
    for k, name in (("self", "self"), ("recv", "recv_count"), ("flags", "flags"),
                    ("c_off", "created_off"), ("c_owner", "created_owner"),
                    ("c_target", "created_target"), ("s_off", "spawned_off"),
                    ("spawned", "spawned"), ("u_off", "updated_off"), ("u_ref", "updated_ref"),
                    ("u_info", "updated_info")):
        a = np.ascontiguousarray(getattr(batch, name))
        keep.append(a)
        setattr(wb, k, a.ctypes.data)
    b = lib.wl_deltas_create()
    try:
        d = WlDeltas()
        lib.wl_deltas_build(b, C.byref(wb), F, dgs, C.byref(d))
        ns, no = d.n_shadows, d.n_out
        out = DeltaBatch(_arr(d.id, ns, np.uint64), _arr(d.recv, ns, np.int32),
                         _arr(d.sup, ns, np.uint64), _arr(d.flags, ns, np.uint8),
                         _arr(d.out_off, ns + 1, np.uint32), _arr(d.out_target, no, np.uint64),
                         _arr(d.out_count, no, np.int32))
        return out, _arr(d.graph_off, d.n_graphs + 1, np.uint32)
    finally:
        lib.wl_deltas_destroy(b)


def undo_of(deltas, location: int):
    """UndoLog.mergeDeltaGraph (UndoLog.java:39-67) over a downed node's merged
    deltas: every shadow the node did not own (not interned) gives back its
    receive count and its created refs.  Fields with nothing left to undo are
    kept, as the reference's admitted map keeps them.  Returns an UndoBatch."""
    from crgc_hip import abi
    from crgc_hip.batch import UndoBatch
    fields = {}
    ext = np.nonzero((deltas.flags & abi.DELTA_INTERNED) == 0)[0]
    for r in ext.tolist():
        a = int(deltas.id[r])
        f = fields.setdefault(a, [0, {}])
        f[0] -= int(deltas.recv_count[r])
        for k in range(int(deltas.out_off[r]), int(deltas.out_off[r + 1])):
            t = int(deltas.out_target[k])
            c = f[1].get(t, 0) - int(deltas.out_count[k])
            if c:
                f[1][t] = c
            else:
                f[1].pop(t, None)
    return UndoBatch.from_fields(location, [(a, m, list(refs.items()))
                                            for a, (m, refs) in fields.items()])
