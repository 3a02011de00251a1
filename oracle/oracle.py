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
    fresh = all(os.path.exists(lib) and os.path.getmtime(lib) >= os.path.getmtime(os.path.join(_HERE, src))
                for lib, src in ((LIB_PATH, "crgc_oracle.cpp"), (OMP_LIB_PATH, "omp_baseline.cpp")))
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


def omp_trace_baseline(g: "OracleGraph", threads: int, reps: int = 3) -> dict:
    """BENCH ONLY: the OpenMP trace (oracle/omp_baseline.cpp) over a CSR snapshot
    of the oracle's graph: best wall seconds of `reps` mark + sweep passes."""
    lib = C.CDLL(OMP_LIB_PATH)
    e = abi.CrgcGraphExport()
    lib_o = g.lib
    lib_o.oracle_export(g.h, C.byref(e))
    nv, ne = int(e.n_vertices), int(e.n_edges)
    ids, rc = np.zeros(nv, np.uint64), np.zeros(nv, np.int32)
    fl, sup = np.zeros(nv, np.uint8), np.zeros(nv, np.uint64)
    eo, et, ec = np.zeros(ne, np.uint64), np.zeros(ne, np.uint64), np.zeros(ne, np.int32)
    e.vertex_cap, e.edge_cap = nv, ne
    e.id, e.recv_count, e.flags, e.supervisor = _ptr(ids), _ptr(rc), _ptr(fl), _ptr(sup)
    e.edge_owner, e.edge_target, e.edge_count = _ptr(eo), _ptr(et), _ptr(ec)
    if lib_o.oracle_export(g.h, C.byref(e)) != abi.OK:
        raise RuntimeError("oracle export failed")
    best = C.c_double()
    out = [C.c_uint64() for _ in range(4)]
    P = C.c_void_p
    lib.omp_trace_bench.argtypes = [C.c_uint64, P, P, P, P, C.c_uint64, P, P, P, C.c_int, C.c_int,
                                    C.POINTER(C.c_double)] + [C.POINTER(C.c_uint64)] * 4
    lib.omp_trace_bench.restype = C.c_int
    if lib.omp_trace_bench(nv, _ptr(ids), _ptr(rc), _ptr(fl), _ptr(sup), ne, _ptr(eo), _ptr(et),
                           _ptr(ec), threads, reps, C.byref(best), *[C.byref(x) for x in out]):
        raise RuntimeError("omp baseline: malformed snapshot")
    return {"seconds": best.value, "edges_scanned": out[0].value, "marked": out[1].value,
            "garbage": out[2].value, "kill": out[3].value, "vertices": nv, "edges": ne}

