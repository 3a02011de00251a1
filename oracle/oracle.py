"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (crgc_oracle.cpp).

The oracle restates the reference's ShadowGraph (ShadowGraph.java) on the CPU.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; the product path (uigc-akka_amd/) never does.

Parity status: pinned by known-answer scenarios restated from the reference's
own integration specs (SupervisionSpec, SimpleActorSpec, SelfMessagingSpec,
ManyMessagesSpec, RandomSpec) and its unit specs (RefobInfoSpec,
SerializationSpec) — see tests/test_oracle_kats.py.  The reference itself
(Java/Scala on a forked Akka) cannot be compiled or run in this pipeline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
sys.path.insert(0, os.path.join(_REPO, "uigc-akka_amd"))
from crgc_hip import abi  # noqa: E402
from crgc_hip.batch import TraceResult, export_to_state, _ptr  # noqa: E402

LIB_PATH = os.path.join(_HERE, "_build", "libcrgc_oracle.so")


OMP_LIB_PATH = os.path.join(_HERE, "_build", "libcrgc_omp.so")


def build(force: bool = False) -> str:
    """Compile the oracle (and the OpenMP bench baseline) with g++ (oracle/Makefile)."""
    hdrs = [os.path.join(_REPO, "include", "crgc.h"), os.path.join(_HERE, "crgc_oracle.h")]
    fresh = all(os.path.exists(lib) and
                all(os.path.getmtime(lib) >= os.path.getmtime(f) for f in [os.path.join(_HERE, src)] + hdrs)
                for lib, src in ((LIB_PATH, "crgc_oracle.cpp"), (OMP_LIB_PATH, "omp_graph.cpp")))
    if not force and fresh:
        return LIB_PATH
    os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return LIB_PATH


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = C.CDLL(LIB_PATH)
        lib.oracle_create.restype = C.c_void_p
        lib.oracle_create.argtypes = [C.c_uint32, C.c_uint32]
        abi._declare(lib, "oracle_")
        _lib = lib
    return _lib


class OracleGraph:
    """Same surface as crgc_hip.ShadowGraph, computed by the CPU restatement."""

    def __init__(self, entry_field_size: int = 4, delta_graph_size: int = 64):
        self.lib = load()
        self.h = self.lib.oracle_create(entry_field_size, delta_graph_size)

    def close(self):
        if self.h:
            self.lib.oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, where):
        if rc != abi.OK:
            raise abi.CrgcError(rc, "oracle." + where)

    def merge_entries(self, batch):
        self._chk(self.lib.oracle_merge_entries(self.h, C.byref(batch.struct())), "merge_entries")

    def merge_deltas(self, batch):
        self._chk(self.lib.oracle_merge_deltas(self.h, C.byref(batch.struct())), "merge_deltas")

    def merge_undo(self, log):
        self._chk(self.lib.oracle_merge_undo(self.h, C.byref(log.struct())), "merge_undo")

    def trace(self, should_kill: bool = True) -> TraceResult:
        n = self.live_count()
        g = np.zeros(max(n, 1), np.uint64)
        k = np.zeros(max(n, 1), np.uint64)
        out = abi.CrgcTraceOut()
        out.garbage_ids, out.garbage_cap = _ptr(g), n
        out.kill_ids, out.kill_cap = _ptr(k), n
        self._chk(self.lib.oracle_trace(self.h, int(bool(should_kill)), C.byref(out)), "trace")
        st = out.stats
        return TraceResult(g[:out.n_garbage].copy(), k[:out.n_kill].copy(), int(out.n_live),
                           st.pseudo_roots, st.edges_scanned, st.sup_edges, st.levels,
                           st.launches)

    def local_roots(self):
        n = C.c_uint64()
        self._chk(self.lib.oracle_local_roots(self.h, None, 0, C.byref(n)), "local_roots")
        buf = np.zeros(max(n.value, 1), np.uint64)
        self._chk(self.lib.oracle_local_roots(self.h, _ptr(buf), n.value, C.byref(n)),
                  "local_roots")
        return buf[:n.value].copy()

    def count_reachable_from(self, location: int) -> int:
        v = C.c_int64()
        self._chk(self.lib.oracle_count_reachable_from(self.h, location, C.byref(v)),
                  "count_reachable_from")
        return v.value

    def total_actors_seen(self) -> int:
        v = C.c_uint64()
        self._chk(self.lib.oracle_total_actors_seen(self.h, C.byref(v)), "total_actors_seen")
        return v.value

    def live_count(self) -> int:
        v = C.c_uint64()
        self._chk(self.lib.oracle_live_count(self.h, C.byref(v)), "live_count")
        return v.value

    def export(self):
        return export_to_state(self.lib.oracle_export, self.h)


class OmpGraph:
    """The strong CPU baseline (oracle/omp_graph.cpp), a parallel OpenMP merge +
    trace over the same entry batches: bench.py times it, and the full-size
    GPU parity tests check the HIP graph against it (its sets are pinned to the
    oracle's by tests/test_omp_graph_cpu.py)."""

    def __init__(self, F: int = 4, vertex_hint: int = 1 << 16, threads: int = 0):
        build()
        lib = C.CDLL(OMP_LIB_PATH)
        lib.omp_graph_create.restype = C.c_void_p
        lib.omp_graph_create.argtypes = [C.c_uint32, C.c_uint64]
        lib.omp_graph_destroy.argtypes = [C.c_void_p]
        lib.omp_graph_merge.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        lib.omp_graph_merge_deltas.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        lib.omp_graph_merge_undo.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        lib.omp_graph_trace.argtypes = ([C.c_void_p, C.c_int, C.c_int] + [C.POINTER(C.c_uint64)] * 5 +
                                        [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64])
        self.lib, self.threads = lib, threads
        self.h = lib.omp_graph_create(F, vertex_hint)
        self._ids = None

    def close(self):
        if self.h:
            self.lib.omp_graph_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def merge_entries(self, batch):
        rc = self.lib.omp_graph_merge(self.h, C.addressof(batch.struct()), self.threads)
        if rc:
            raise abi.CrgcError(rc, "omp_graph_merge")

    def merge_deltas(self, batch):
        """N x ShadowGraph.mergeDelta (DeltaBatch in host memory)."""
        rc = self.lib.omp_graph_merge_deltas(self.h, C.addressof(batch.struct()), self.threads)
        if rc:
            raise abi.CrgcError(rc, "omp_graph_merge_deltas")

    def merge_undo(self, log):
        """ShadowGraph.mergeUndoLog (UndoBatch in host memory); CRGC_E_UNDO_NEW_SHADOW
        is the reference's ConcurrentModificationException, the graph unchanged."""
        rc = self.lib.omp_graph_merge_undo(self.h, C.addressof(log.struct()), self.threads)
        if rc:
            raise abi.CrgcError(rc, "omp_graph_merge_undo")

    def trace(self, should_kill: bool = True, ids: bool = False) -> dict:
        """Counts; with ids=True also 'garbage_ids' / 'kill_ids' (unsorted)."""
        v = [C.c_uint64() for _ in range(5)]
        g = k = None
        if ids:
            if self._ids is None:
                self.reserve_ids(1 << 16)
            g, k = self._ids
        rc = self.lib.omp_graph_trace(self.h, int(should_kill), self.threads, *[C.byref(x) for x in v],
                                      g.ctypes.data if ids else None, len(g) if ids else 0,
                                      k.ctypes.data if ids else None, len(k) if ids else 0)
        if rc == abi.E2BIG:  # the trace happened (counts exact): the ids of this one are lost
            self.reserve_ids(2 * int(max(v[0].value, v[1].value)) + 1024)
            raise abi.CrgcError(rc, "omp_graph_trace: id buffers too small (grown for the next trace)")
        if rc:
            raise abi.CrgcError(rc, "omp_graph_trace")
        out = dict(zip(("garbage", "kill", "live", "edges_scanned", "pseudo_roots"), (x.value for x in v)))
        if ids:
            out["garbage_ids"] = g[:out["garbage"]].copy()
            out["kill_ids"] = k[:out["kill"]].copy()
        return out

    def reserve_ids(self, n: int):
        """Id buffers for traces of up to n garbage shadows."""
        self._ids = (np.zeros(n, np.uint64), np.zeros(n, np.uint64))
