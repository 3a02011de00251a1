"""The C++ C5 stream builders (workload/deltas.cpp, world.undo_of) against the
Python restatements of DeltaGraph / UndoLog (workload/delta.py), on CPU."""
import numpy as np

import delta
import world
from crgc_hip import DeltaBatch

FIELDS = ("id", "recv_count", "supervisor", "flags", "out_off", "out_target", "out_count")


def _batches():
    w = world.World(seed=3, location=2)
    w.bulk_graph(3000, 30000, alpha=2.1, n_roots=30)
    yield w.take(20000)            # spawn tree + acquaintance edges
    yield w.wakeup_batch(5000)     # sends, shares, releases, receives


def test_cpp_delta_builder_matches_python_restatement():
    for b in _batches():
        d, graph_off = world.deltas_of(b)
        gs = delta.deltas_from_entries(b.to_entries(), address=2)
        ref = DeltaBatch.concat([g.to_batch() for g in gs])
        assert len(graph_off) - 1 == len(gs)
        assert list(np.diff(graph_off)) == [g.size for g in gs]
        for k in FIELDS:
            assert np.array_equal(getattr(d, k), getattr(ref, k)), k


def _canon(u):
    out = {}
    for i, a in enumerate(u.actor.tolist()):
        refs = {int(t): int(c) for t, c in zip(u.created_target[u.created_off[i]:u.created_off[i + 1]],
                                               u.created_count[u.created_off[i]:u.created_off[i + 1]])}
        out[a] = (int(u.message_count[i]), refs)
    return out


def test_undo_of_matches_python_undo_log():
    for b in _batches():
        d, _ = world.deltas_of(b)
        log = delta.UndoLog(2)
        for g in delta.deltas_from_entries(b.to_entries(), address=2):
            log.mergeDeltaGraph(g)
        assert _canon(world.undo_of(d, 2)) == _canon(log.to_batch())
