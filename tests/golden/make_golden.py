"""Generate tests/golden/*.npz: seeded input streams + the oracle's outputs.

The reference (Java/Scala on a forked Akka) cannot run in this pipeline and
ships no ShadowGraph vectors, so these fixtures are produced by
the CPU oracle (oracle/crgc_oracle.cpp), itself pinned by the reference-spec
KATs (tests/kats.py).  They freeze the inputs and expected outputs so that
both the oracle and the HIP path are checked against stored data rather than
against a generator that might drift.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for sub in ("uigc-akka_amd", "workload", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, sub))

import fuzz  # noqa: E402
import kats  # noqa: E402
import oracle  # noqa: E402

ENTRY_FIELDS = ("self", "recv_count", "flags", "created_off", "created_owner", "created_target",
                "spawned_off", "spawned", "updated_off", "updated_ref", "updated_info")
DELTA_FIELDS = ("id", "recv_count", "supervisor", "flags", "out_off", "out_target", "out_count")
UNDO_FIELDS = ("actor", "message_count", "created_off", "created_target", "created_count")


def record(steps_iter, path):
    """steps_iter yields ("E"|"D"|"U", batch) or ("T",); the oracle runs them."""
    o = oracle.OracleGraph()
    arrs = {}
    kinds = []
    for i, st in enumerate(steps_iter(o)):
        kind = st[0]
        kinds.append(kind)
        if kind == "E":
            o.merge_entries(st[1])
            for f in ENTRY_FIELDS:
                arrs[f"{i}_{f}"] = getattr(st[1], f)
        elif kind == "D":
            o.merge_deltas(st[1])
            for f in DELTA_FIELDS:
                arrs[f"{i}_{f}"] = getattr(st[1], f)
        elif kind == "U":
            o.merge_undo(st[1])
            arrs[f"{i}_location"] = np.array([st[1].node_location], np.uint16)
            for f in UNDO_FIELDS:
                arrs[f"{i}_{f}"] = getattr(st[1], f)
        else:
            r = o.trace(True)
            arrs[f"{i}_garbage"] = np.sort(r.garbage)
            arrs[f"{i}_kill"] = np.sort(r.kill)
            arrs[f"{i}_live"] = np.array([r.n_live], np.int64)
            arrs[f"{i}_roots"] = np.array([r.pseudo_roots], np.int64)
    arrs["kinds"] = np.array([ord(k) for k in kinds], np.uint8)
    arrs["total_actors_seen"] = np.array([o.total_actors_seen()], np.int64)
    np.savez_compressed(path, **arrs)
    print(path, os.path.getsize(path), "bytes,", len(kinds), "steps")


def fuzz_steps(seed, n_steps=10):
    def gen(o):
        fz = fuzz.Fuzz(seed)
        for step in range(n_steps):
            yield ("E", fz.entries(150 + 40 * step))
            if step % 2 == 1:
                yield ("D", fz.deltas(4))
            if step == 7:
                yield ("U", fz.undo(o.export().vertices.keys()))
            yield ("T",)
            fz.sync(o.export())
    return gen


def random_spec_steps(seed, max_actors):
    def gen(o):
        w = kats.RandomWorld(seed, max_actors, wake_every=20)
        for batch in w.steps():
            yield ("E", batch)
            yield ("T",)
    return gen


if __name__ == "__main__":
    oracle.build()
    record(fuzz_steps(101), os.path.join(HERE, "fuzz_s101.npz"))
    record(fuzz_steps(202), os.path.join(HERE, "fuzz_s202.npz"))
    record(random_spec_steps(303, 500), os.path.join(HERE, "random_spec_s303.npz"))
