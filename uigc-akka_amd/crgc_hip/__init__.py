"""crgc_hip — MI355X-native CRGC garbage-detection hot path.

The product is the C-ABI shared library built from ../csrc (libcrgc_hip.so,
HIP kernels for gfx950); this package is its host-side mirror of the reference
ShadowGraph surface (ShadowGraph.java), bound through ctypes.
"""
from . import abi
from .batch import Entry, EntryBatch, DeltaBatch, UndoBatch, TraceResult, RefobInfo, GraphState, HostArena
from .graph import HostCollectives, ShadowGraph, ShardedShadowGraph, Transport, UndoAccumulator, shard_of

__all__ = ["abi", "Entry", "EntryBatch", "HostArena", "DeltaBatch", "UndoBatch", "TraceResult", "RefobInfo",
           "GraphState", "HostCollectives", "ShadowGraph", "ShardedShadowGraph", "Transport", "UndoAccumulator",
           "shard_of"]
