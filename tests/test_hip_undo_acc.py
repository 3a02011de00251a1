"""UndoLog folding on the device (crgc_undo_acc) against the
host restatement of UndoLog (workload/delta.py: UndoLog.java:39-104) and the
oracle's mergeUndoLog.  An UndoLog is compared as a map: actor -> (message
count, created refs with nonzero counts) — absent == 0 (UndoLog.java:95-104),
field order unspecified."""
import numpy as np
import pytest

import cluster
import world
from crgc_hip import UndoBatch, abi

pytestmark = pytest.mark.gpu


def _canon(u: UndoBatch):
    out = {}
    for i, a in enumerate(u.actor.tolist()):
        lo, hi = int(u.created_off[i]), int(u.created_off[i + 1])
        refs = {int(t): int(c) for t, c in zip(u.created_target[lo:hi], u.created_count[lo:hi]) if c}
        assert int(a) not in out
        out[int(a)] = (int(u.message_count[i]), refs)
    return out


def _fold(acc, cw, merged, downed):
    """What node 1's collector folds for `downed`: its DeltaGraphs on arrival
    (LocalGC.scala:133) and the ingress entries admitted from it."""
    for k, dg in merged:
        if k == downed:
            acc.fold_deltas(dg.to_batch())
    for (sk, _), ie in cw.ingress.items():
        if sk == downed:
            fields = [(a, f.messageCount, list(f.createdRefs.items()))
                      for a, f in ie.admitted.items()]
            acc.fold_ingress(UndoBatch.from_fields(0, fields))


def _cluster_run(seed, turns=6):
    cw = cluster.ClusterWorld(seed=seed, n_nodes=8, max_actors=2000)
    merged = []
    for _ in range(turns):
        cw.run_turns(400)
        _, deltas = cw.flush(0)
        merged.extend(deltas)
    return cw, merged


@pytest.mark.parametrize("seed", [3, 4])
def test_fold_deltas_and_ingress_match_undo_log(hip_mod, seed):
    cw, merged = _cluster_run(seed)
    g = hip_mod.ShadowGraph()
    for downed in (6, 7):
        acc = g.undo_accumulator(downed + 1)
        _fold(acc, cw, merged, downed)
        want = cw.undo_log(downed, merged).to_batch()
        assert _canon(acc.export()) == _canon(want)
        acc.close()


def test_growth_and_device_batches(hip_mod):
    """Many folds from 4096-slot tables: rehashing as the log grows; device-resident input."""
    g = hip_mod.ShadowGraph()
    w = world.World(seed=21, location=4)
    w.bulk_graph(50_000, 400_000, alpha=2.1, n_roots=100)
    acc = g.undo_accumulator(4)
    want = {}
    for i, b in enumerate(w.batches(1 << 15)):
        d, _ = world.deltas_of(b)
        acc.fold_deltas(d.to_device() if i % 2 else d)
        for a, (m, refs) in _canon(world.undo_of(d, 4)).items():
            pm, pr = want.get(a, (0, {}))
            for t, c in refs.items():
                pr[t] = pr.get(t, 0) + c
                if pr[t] == 0:
                    del pr[t]
            want[a] = (pm + m, pr)
    assert len(want) > 4096
    assert _canon(acc.export()) == want


def test_merge_undo_acc_matches_oracle(hip_mod, oracle_mod):
    """ShadowGraph.mergeUndoLog with the device-folded log: the graph afterwards
    (or the CME, E11) equals the oracle's with the host-built log."""
    from crgc_hip import DeltaBatch  # noqa: F401
    for seed in (5, 6, 8):
        cw, merged = _cluster_run(seed, turns=5)
        g, o = hip_mod.ShadowGraph(), oracle_mod.OracleGraph()
        for k, dg in merged:
            b = dg.to_batch()
            g.merge_deltas(b)
            o.merge_deltas(b)
        downed = 7
        acc = g.undo_accumulator(downed + 1)
        _fold(acc, cw, merged, downed)
        log = cw.undo_log(downed, merged).to_batch()
        try:
            o.merge_undo(log)
            want = None
        except abi.CrgcError as e:
            want = e.code
        if want is None:
            g.merge_undo_acc(acc)
            assert g.export() == o.export()
            assert g.count_reachable_from(downed + 1) == o.count_reachable_from(downed + 1)
        else:
            with pytest.raises(abi.CrgcError) as e:
                g.merge_undo_acc(acc)
            assert e.value.code == want
        acc.close()
