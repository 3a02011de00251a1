"""ctypes mirror of include/crgc.h (the C ABI of the HIP shadow graph).

The struct layouts here must match include/crgc.h field for field; the
`test_abi_layout` test checks the sizes against the C compiler's view.
"""
from __future__ import annotations

import ctypes as C
import os

ABI_VERSION = 5

OK = 0
E_INVAL = -1
E_NOMEM = -2
E_DEVICE = -3
E2BIG = -4
E_NULL_SUPERVISOR = -5
E_UNDO_NEW_SHADOW = -6
E_POISONED = -7
E_TIMEOUT = -8

NO_ACTOR = 0xFFFFFFFFFFFFFFFF
DEAD_ACTOR = 0xFFFFFFFFFFFFFFFE

MEM_HOST = 0
MEM_DEVICE = 1

F_INTERNED = 0x02
F_LOCAL = 0x04
F_BUSY = 0x08
F_ROOT = 0x10
F_HALTED = 0x20
F_PROXY = 0x40

ENTRY_BUSY = 0x01
ENTRY_ROOT = 0x02
DELTA_INTERNED = 0x01
DELTA_ROOT = 0x02
DELTA_BUSY = 0x04

_P = C.c_void_p
_U64 = C.c_uint64


class CrgcConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32),
        ("device", C.c_int32),
        ("entry_field_size", C.c_uint32),
        ("delta_graph_size", C.c_uint32),
        ("vertex_capacity", _U64),
        ("edge_capacity", _U64),
        ("stream", _P),
        ("n_shards", C.c_uint32),
        ("shard", C.c_uint32),
        ("transport", _P),
        ("proxy_capacity", _U64),
    ]


class CrgcEntryBatch(C.Structure):
    _fields_ = [
        ("n_entries", _U64),
        ("self", _P),
        ("recv_count", _P),
        ("flags", _P),
        ("created_off", _P),
        ("created_owner", _P),
        ("created_target", _P),
        ("spawned_off", _P),
        ("spawned", _P),
        ("updated_off", _P),
        ("updated_ref", _P),
        ("updated_info", _P),
        ("memory", C.c_uint32),
    ]


class CrgcDeltaBatch(C.Structure):
    _fields_ = [
        ("n_shadows", _U64),
        ("id", _P),
        ("recv_count", _P),
        ("supervisor", _P),
        ("flags", _P),
        ("out_off", _P),
        ("out_target", _P),
        ("out_count", _P),
        ("memory", C.c_uint32),
    ]


class CrgcUndoLog(C.Structure):
    _fields_ = [
        ("node_location", C.c_uint16),
        ("_pad", C.c_uint16 * 3),
        ("n_fields", _U64),
        ("actor", _P),
        ("message_count", _P),
        ("created_off", _P),
        ("created_target", _P),
        ("created_count", _P),
        ("memory", C.c_uint32),
    ]


class CrgcTraceStats(C.Structure):
    _fields_ = [
        ("pseudo_roots", _U64),
        ("edges_scanned", _U64),
        ("sup_edges", _U64),
        ("levels", _U64),
        ("launches", _U64),
        ("ms_mark", C.c_double),
        ("ms_sweep", C.c_double),
        ("ms_total", C.c_double),
        ("ms_frontier", C.c_double),
        ("ms_tail", C.c_double),
        ("ms_expand", C.c_double),
        ("rounds", _U64),
        ("ids_sent", _U64),
        ("ms_exchange", C.c_double),
        ("expand_launches", _U64),
        ("expand_bytes", _U64),
        ("exchange_bytes", _U64),
        ("time_query_failures", _U64),
        ("direct_lists", _U64),
    ]


class CrgcTraceOut(C.Structure):
    _fields_ = [
        ("garbage_ids", _P),
        ("garbage_cap", _U64),
        ("n_garbage", _U64),
        ("kill_ids", _P),
        ("kill_cap", _U64),
        ("n_kill", _U64),
        ("n_live", _U64),
        ("stats", CrgcTraceStats),
    ]


class CrgcGraphExport(C.Structure):
    _fields_ = [
        ("vertex_cap", _U64),
        ("n_vertices", _U64),
        ("id", _P),
        ("recv_count", _P),
        ("flags", _P),
        ("supervisor", _P),
        ("edge_cap", _U64),
        ("n_edges", _U64),
        ("edge_owner", _P),
        ("edge_target", _P),
        ("edge_count", _P),
    ]


class CrgcDeltaGraphs(C.Structure):
    _fields_ = [
        ("memory", C.c_uint32),
        ("_pad", C.c_uint32),
        ("graph_cap", _U64),
        ("n_graphs", _U64),
        ("graph_off", _P),
        ("wire_off", _P),
        ("shadow_cap", _U64),
        ("n_shadows", _U64),
        ("id", _P),
        ("recv_count", _P),
        ("supervisor", _P),
        ("flags", _P),
        ("out_off", _P),
        ("out_cap", _U64),
        ("n_out", _U64),
        ("out_target", _P),
        ("out_count", _P),
        ("wire_cap", _U64),
        ("wire_bytes", _U64),
        ("wire", _P),
    ]


class CrgcUndoLogOut(C.Structure):
    _fields_ = [
        ("field_cap", _U64),
        ("n_fields", _U64),
        ("actor", _P),
        ("message_count", _P),
        ("created_off", _P),
        ("created_cap", _U64),
        ("n_created", _U64),
        ("created_target", _P),
        ("created_count", _P),
    ]


# crgc_host_collectives (include/crgc.h): the caller's host collectives
HOST_ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_size_t)
HOST_ALLTOALLV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.POINTER(C.c_size_t),
                             C.POINTER(C.c_size_t), C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t))


class CrgcUsage(C.Structure):
    _fields_ = [(n, _U64) for n in ("slot_top", "slot_cap", "proxy_top", "proxy_cap", "free_slots",
                                   "pool_top", "pool_cap", "etab_used", "etab_cap",
                                   "rebuilds", "grows", "repacks")]


class HostCollectives(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("allgather", HOST_ALLGATHER), ("alltoallv", HOST_ALLTOALLV)]


# Entry points declared in include/crgc.h — every one must be exported.
EXPORTED_SYMBOLS = (
    "crgc_create",
    "crgc_destroy",
    "crgc_merge_entries",
    "crgc_merge_entries_async",
    "crgc_merge_deltas",
    "crgc_merge_undo",
    "crgc_trace",
    "crgc_last_trace",
    "crgc_local_roots",
    "crgc_count_reachable_from",
    "crgc_total_actors_seen",
    "crgc_live_count",
    "crgc_compact",
    "crgc_sync",
    "crgc_export",
    "crgc_build_delta_graphs",
    "crgc_undo_acc_create",
    "crgc_undo_acc_destroy",
    "crgc_undo_acc_fold_deltas",
    "crgc_undo_acc_fold_ingress",
    "crgc_undo_acc_export",
    "crgc_merge_undo_acc",
    "crgc_strerror",
    "crgc_last_error_detail",
    "crgc_transport_rccl_id",
    "crgc_transport_rccl",
    "crgc_transport_local",
    "crgc_transport_host",
    "crgc_transport_destroy",
    "crgc_shard_of",
    "crgc_host_register",
    "crgc_host_unregister",
    "crgc_usage_of",
)


def _declare(lib: C.CDLL, prefix: str) -> None:
    """Attach argtypes/restypes for the `prefix`-named entry points."""
    P = C.POINTER
    g = _P
    sig = {
        "merge_entries": (C.c_int, [g, P(CrgcEntryBatch)]),
        "merge_deltas": (C.c_int, [g, P(CrgcDeltaBatch)]),
        "merge_undo": (C.c_int, [g, P(CrgcUndoLog)]),
        "trace": (C.c_int, [g, C.c_int, P(CrgcTraceOut)]),
        "local_roots": (C.c_int, [g, _P, _U64, P(_U64)]),
        "count_reachable_from": (C.c_int, [g, C.c_uint16, P(C.c_int64)]),
        "total_actors_seen": (C.c_int, [g, P(_U64)]),
        "live_count": (C.c_int, [g, P(_U64)]),
        "export": (C.c_int, [g, P(CrgcGraphExport)]),
        "destroy": (None, [g]),
    }
    if prefix == "crgc_":  # product-only entry points (the JVM compacts by itself; drain-loop chunks)
        sig["compact"] = (C.c_int, [g])
        sig["sync"] = (C.c_int, [g])
        sig["merge_entries_async"] = (C.c_int, [g, P(CrgcEntryBatch)])
        if hasattr(lib, "crgc_usage_of") or not os.environ.get("CRGC_LIB_AB"):  # an A/B build may predate it
            sig["usage_of"] = (C.c_int, [g, P(CrgcUsage)])
    for name, (res, args) in sig.items():
        fn = getattr(lib, prefix + name)
        fn.restype = res
        fn.argtypes = args


_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libcrgc_hip.so")

_lib = None


def load_library(path: str | None = None) -> C.CDLL:
    """Load the HIP shim.  Fails loudly: there is no CPU fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("CRGC_LIB_AB") or LIB_PATH  # CRGC_LIB_AB: A/B of two builds
    if not os.path.exists(p):
        raise RuntimeError(
            f"libcrgc_hip.so not found at {p}; build it with "
            "`python __graft_entry__.py build` (hipcc --offload-arch=gfx950)")
    lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
    lib.crgc_create.restype = C.c_int
    lib.crgc_create.argtypes = [C.POINTER(CrgcConfig), C.POINTER(_P)]
    lib.crgc_last_trace.restype = C.c_int
    lib.crgc_last_trace.argtypes = [_P, C.POINTER(CrgcTraceOut)]
    lib.crgc_strerror.restype = C.c_char_p
    lib.crgc_strerror.argtypes = [C.c_int]
    if hasattr(lib, "crgc_last_error_detail"):  # an A/B build may predate it
        lib.crgc_last_error_detail.restype = C.c_char_p
        lib.crgc_last_error_detail.argtypes = []
    lib.crgc_transport_rccl_id.restype = C.c_int
    lib.crgc_transport_rccl_id.argtypes = [C.c_char_p]
    lib.crgc_transport_rccl.restype = C.c_int
    lib.crgc_transport_rccl.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.c_int32,
                                        C.POINTER(_P)]
    lib.crgc_transport_local.restype = C.c_int
    lib.crgc_transport_local.argtypes = [C.c_uint32, C.POINTER(_P)]
    if hasattr(lib, "crgc_transport_host"):
        lib.crgc_transport_host.restype = C.c_int
        lib.crgc_transport_host.argtypes = [C.POINTER(HostCollectives), C.c_uint32, C.c_uint32, C.c_int32,
                                            C.POINTER(_P)]
    lib.crgc_transport_destroy.restype = None
    lib.crgc_transport_destroy.argtypes = [_P]
    lib.crgc_shard_of.restype = C.c_uint32
    lib.crgc_shard_of.argtypes = [_U64, C.c_uint32]
    lib.crgc_undo_acc_create.restype = C.c_int
    lib.crgc_undo_acc_create.argtypes = [_P, C.c_uint16, C.POINTER(_P)]
    lib.crgc_undo_acc_destroy.restype = None
    lib.crgc_undo_acc_destroy.argtypes = [_P]
    lib.crgc_undo_acc_fold_deltas.restype = C.c_int
    lib.crgc_undo_acc_fold_deltas.argtypes = [_P, C.POINTER(CrgcDeltaBatch)]
    lib.crgc_undo_acc_fold_ingress.restype = C.c_int
    lib.crgc_undo_acc_fold_ingress.argtypes = [_P, C.POINTER(CrgcUndoLog)]
    lib.crgc_undo_acc_export.restype = C.c_int
    lib.crgc_undo_acc_export.argtypes = [_P, C.POINTER(CrgcUndoLogOut)]
    lib.crgc_merge_undo_acc.restype = C.c_int
    lib.crgc_merge_undo_acc.argtypes = [_P, _P]
    if hasattr(lib, "crgc_host_register") or not os.environ.get("CRGC_LIB_AB"):  # an A/B build may predate it
        lib.crgc_host_register.restype = C.c_int
        lib.crgc_host_register.argtypes = [_P, _P, _U64]
        lib.crgc_host_unregister.restype = C.c_int
        lib.crgc_host_unregister.argtypes = [_P, _P]
    lib.crgc_build_delta_graphs.restype = C.c_int
    lib.crgc_build_delta_graphs.argtypes = [_P, C.POINTER(CrgcEntryBatch), C.POINTER(CrgcDeltaGraphs)]
    _declare(lib, "crgc_")
    if path is None:
        _lib = lib
    return lib


class CrgcError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str = ""):
        self.code = code
        self.detail = detail
        super().__init__(f"{where}: {code} ({ERROR_NAMES.get(code, '?')})"
                         + (f" at {detail}" if detail else ""))


def last_error_detail() -> str:
    """crgc_last_error_detail(): where this thread's last failed call went wrong."""
    if _lib is None or not hasattr(_lib, "crgc_last_error_detail"):
        return ""
    return (_lib.crgc_last_error_detail() or b"").decode(errors="replace")


ERROR_NAMES = {
    OK: "OK",
    E_INVAL: "CRGC_E_INVAL",
    E_NOMEM: "CRGC_E_NOMEM",
    E_DEVICE: "CRGC_E_DEVICE",
    E2BIG: "CRGC_E2BIG",
    E_NULL_SUPERVISOR: "CRGC_E_NULL_SUPERVISOR",
    E_UNDO_NEW_SHADOW: "CRGC_E_UNDO_NEW_SHADOW",
    E_POISONED: "CRGC_E_POISONED",
    E_TIMEOUT: "CRGC_E_TIMEOUT",
}
