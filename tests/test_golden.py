"""Replay the committed golden streams (tests/golden/*.npz, made by
tests/golden/make_golden.py) through the oracle (CPU) and the HIP path (GPU)
and compare with the stored garbage / kill sets and live counts."""
import glob
import os

import numpy as np
import pytest

from crgc_hip.batch import DeltaBatch, EntryBatch, UndoBatch

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))
ENTRY_FIELDS = ("self", "recv_count", "flags", "created_off", "created_owner", "created_target",
                "spawned_off", "spawned", "updated_off", "updated_ref", "updated_info")
DELTA_FIELDS = ("id", "recv_count", "supervisor", "flags", "out_off", "out_target", "out_count")
UNDO_FIELDS = ("actor", "message_count", "created_off", "created_target", "created_count")


def replay(graph, path):
    z = np.load(path)  # allow_pickle=False (default)
    for i, k in enumerate(z["kinds"].tolist()):
        k = chr(k)
        if k == "E":
            graph.merge_entries(EntryBatch(*(z[f"{i}_{f}"] for f in ENTRY_FIELDS)))
        elif k == "D":
            graph.merge_deltas(DeltaBatch(*(z[f"{i}_{f}"] for f in DELTA_FIELDS)))
        elif k == "U":
            graph.merge_undo(UndoBatch(int(z[f"{i}_location"][0]),
                                       *(z[f"{i}_{f}"] for f in UNDO_FIELDS)))
        else:
            r = graph.trace(True)
            assert np.array_equal(np.sort(r.garbage), z[f"{i}_garbage"]), f"step {i}"
            assert np.array_equal(np.sort(r.kill), z[f"{i}_kill"]), f"step {i}"
            assert r.n_live == int(z[f"{i}_live"][0])
            assert r.pseudo_roots == int(z[f"{i}_roots"][0])
    assert graph.total_actors_seen() == int(z["total_actors_seen"][0])


def test_fixtures_exist():
    assert len(FIXTURES) >= 3


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_golden_oracle(oracle_mod, path):
    replay(oracle_mod.OracleGraph(), path)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_golden_hip(hip_mod, path):
    replay(hip_mod.ShadowGraph(), path)
