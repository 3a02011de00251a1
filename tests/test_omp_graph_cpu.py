"""The strong CPU baseline (oracle/omp_graph.cpp) computes what the oracle
computes: per wakeup, the same garbage and kill SETS and the same live /
pseudo-root / traced-edge counts on the C1 stream and a C2-shaped one.  This
pins it, so bench.py's cpu_baseline times the same work as the GPU line and the
full-size GPU parity tests (tests/test_hip_full_size.py) may use it as the
checker where the single-thread oracle would take too long."""
import pytest

import world


def _c1():
    w = world.World(seed=0x5EED + 1)
    w.set_mix(send=0.2, share=0.2, release=0.2, spawn=0.2, actions_per_msg=2.0)
    w.uniform_graph(50_000, mean_acq=8.0, n_roots=500, dead_frac=0.05)
    return w, 50_000


def _c2():
    w = world.World(seed=0x5EED + 2)
    w.bulk_graph(50_000, 500_000, alpha=2.1, n_roots=50, cap=100000)
    return w, 50_000


@pytest.mark.parametrize("make", [_c1, _c2], ids=["c1", "c2"])
def test_omp_graph_matches_oracle(oracle_mod, make):
    w, V = make()
    o, p = oracle_mod.OracleGraph(), oracle_mod.OmpGraph(threads=4)
    for b in w.batches(1 << 16):
        o.merge_entries(b)
        p.merge_entries(b)
    for k in range(5):
        if k:
            b = w.wakeup(V // 10, busy=V * 9 // 100, pending=V // 100)
            o.merge_entries(b)
            p.merge_entries(b)
        ro, rp = o.trace(True), p.trace(True, ids=True)
        assert (len(ro.garbage), len(ro.kill), ro.n_live, ro.pseudo_roots, ro.edges_scanned) == \
            (rp["garbage"], rp["kill"], rp["live"], rp["pseudo_roots"], rp["edges_scanned"]), k
        assert ro.garbage_set() == set(rp["garbage_ids"].tolist()), k
        assert ro.kill_set() == set(rp["kill_ids"].tolist()), k
