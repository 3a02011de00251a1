"""Every trace tuning switch gives the oracle's result (HIP vs oracle).

The level kernels read A/B switches per trace (CRGC_* in crgc_api.hip
run_levels).  They change how the mark is computed — push or pull per level,
the narrow-frontier takeover — never what is marked.  (Round 1's losing
variants were removed from the product; profiles/r1h, r1n, r1r keep their A/B.)  Each variant
replays the same seeded stream (a C1-sized power-law graph, then mutator
wakeups) into a fresh graph and must match the oracle wakeup by wakeup.
"""
import pytest

import world

pytestmark = pytest.mark.gpu

ACTORS, EDGES, BATCH, WAKEUPS = 100_000, 1_000_000, 10_000, 3

VARIANTS = [
    {},
    {"CRGC_ALPHA": "0"},                  # round-1 rule: the current frontier's size
    {"CRGC_ALPHA": "0", "CRGC_PULL_CUR_DIV": "0"},  # direction from the previous frontier only
    {"CRGC_ALPHA": "1000000"},            # pull on every dense level, level 0 included
    {"CRGC_PULL": "0"},                   # push only
    {"CRGC_TAIL": "0"},                   # no narrow-frontier takeover
    {"CRGC_TAIL_START": "1000000", "CRGC_TAIL_MAX": "64"},  # early takeover, frequent bails
    {"CRGC_BIN_MIN_SLOTS": "0"},          # the pseudo-root level binned at this size too
    {"CRGC_BIN": "0"},                    # the pseudo-root level's direct push
    {"CRGC_CBITS": "0"},                  # a pull level's finds as candidate bytes (round-4 form)
    {"CRGC_ROOTS_CO": "0"},               # the pseudo-root pass's per-lane 128-B count loads
    {"CRGC_PULL_PRED": "1"},              # the previous trace's pull levels pull again
    {"CRGC_SUPBIN": "0"},                 # binned level 0: supervisor candidate bytes stored at once
    {"CRGC_BIN512": "1", "CRGC_BIN_MIN_SLOTS": "0"},  # binned level 0 with up to 512 bins of 2^16
    # candidate bits after every pull (level 0 included) with frequent k_tail bails
    {"CRGC_ALPHA": "1000000", "CRGC_TAIL_START": "1000000", "CRGC_TAIL_MAX": "64"},
    # k_tail bounded by edge volume: no takeover of a frontier with more out-edges,
    # and a walk whose round reaches hubs with more hands them back (round 6)
    {"CRGC_TAIL_EDGES": "64"},
    {"CRGC_TAIL_EDGES": "256", "CRGC_TAIL_START": "1000000", "CRGC_TAIL_MAX": "65536"},
]


def _stream():
    w = world.World(seed=0x5EED + 11)
    w.bulk_graph(ACTORS, EDGES, alpha=2.1, n_roots=ACTORS // 100)
    return w


def _key(r):
    return (r.garbage_set(), r.kill_set(), r.n_live, r.pseudo_roots, r.sup_edges, r.edges_scanned)


@pytest.fixture(scope="module")
def oracle_results(oracle_mod):
    w = _stream()
    o = oracle_mod.OracleGraph()
    for b in w.batches(1 << 20):
        o.merge_entries(b)
    out = [_key(o.trace(True))]
    for _ in range(WAKEUPS):
        o.merge_entries(w.wakeup_batch(BATCH))
        out.append(_key(o.trace(True)))
    return out


@pytest.mark.parametrize("env", VARIANTS, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()) or "defaults")
def test_trace_switches_match_oracle(hip_mod, oracle_results, monkeypatch, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    w = _stream()
    h = hip_mod.ShadowGraph(vertex_capacity=ACTORS * 2, edge_capacity=EDGES * 2)
    for b in w.batches(1 << 20):
        h.merge_entries(b)
    assert _key(h.trace(True)) == oracle_results[0]
    for i in range(WAKEUPS):
        h.merge_entries(w.wakeup_batch(BATCH).to_device())
        assert _key(h.trace(True)) == oracle_results[i + 1], f"wakeup {i}"


@pytest.mark.parametrize("env", [{}, {"CRGC_BIN_MIN_SLOTS": "0"}, {"CRGC_BIN_MIN_SLOTS": "0", "CRGC_CBITS": "0"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()) or "defaults")
def test_host_batches_binned_level0_match_oracle(hip_mod, oracle_results, monkeypatch, env):
    """Wakeups merged from pageable host memory: the trace's level grids and
    level-0 bins are then sized from an upper bound of slot_top (the batch's
    possible new ids), so bins past the slots in use exist — k_bin_apply must
    store nothing for them (round 5: a bitmap store sized hi - lo faulted
    there when hi < lo)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    w = _stream()
    h = hip_mod.ShadowGraph(vertex_capacity=ACTORS * 2, edge_capacity=EDGES * 2)
    for b in w.batches(1 << 20):
        h.merge_entries(b)
    assert _key(h.trace(True)) == oracle_results[0]
    for i in range(WAKEUPS):
        h.merge_entries(w.wakeup_batch(BATCH))
        assert _key(h.trace(True)) == oracle_results[i + 1], f"wakeup {i}"


def test_sampled_timing_matches_oracle(hip_mod, oracle_results, monkeypatch):
    """CRGC_TIMING_EVERY=2 (round 6): only every other trace carries timing
    events; the traces in between report no device times and no timed
    launches.  What is marked never depends on it."""
    monkeypatch.setenv("CRGC_TIMING_EVERY", "2")
    w = _stream()
    h = hip_mod.ShadowGraph(vertex_capacity=ACTORS * 2, edge_capacity=EDGES * 2)
    for b in w.batches(1 << 20):
        h.merge_entries(b)
    rs = [h.trace(True)]
    assert _key(rs[0]) == oracle_results[0]
    for i in range(WAKEUPS):
        h.merge_entries(w.wakeup_batch(BATCH).to_device())
        rs.append(h.trace(True))
        assert _key(rs[-1]) == oracle_results[i + 1], f"wakeup {i}"
    for k, r in enumerate(rs):
        if k % 2 == 0:
            assert r.ms_mark > 0 and r.expand_launches > 0, k
        else:
            assert r.ms_mark == 0 and r.ms_sweep == 0 and r.expand_launches == 0, k
