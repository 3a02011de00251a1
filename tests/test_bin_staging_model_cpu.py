"""The LDS staging protocol of k_bin_place (crgc_trace.hip bin_try_flush and
the put lambda), modelled step by step under random interleavings of many
writers: every staged position must reach its slice exactly once in value (a
position may be stored twice, with the same target), whatever the order of
exchanges, group flushes, evictions and the final flush.  Each model step is
one atomic LDS / memory operation of the kernel (8-B reads and exchanges).
The round-4 form that stored a group from a second, unverified read loses
entries here (and lost them on the GPU: test_large_host_batches_chunked_and_registered).
"""
import random

import pytest

R, GRP = 32, 16
def run(seed, n_items=400, n_workers=24):
    rnd = random.Random(seed)
    ring = [0] * R          # entry = (pos+1) << 32 | target ; 0 empty
    lc = 0
    glob = {}               # slice position -> set of values written
    targets = list(range(1000, 1000 + n_items))
    # each worker = generator of atomic steps
    def writer(t):
        nonlocal lc
        pos = lc; lc += 1; yield
        s = pos % R
        new = ((pos + 1) << 32) | t
        old = ring[s]; ring[s] = new; yield          # atomic exchange
        if old:
            glob.setdefault((old >> 32) - 1, set()).add(old & 0xFFFFFFFF); yield
        if pos % GRP == GRP - 1:
            g0 = pos - (GRP - 1); s0 = g0 % R
            for attempt in range(4):
                allok = True
                for q in range(0, GRP, 4):
                    es = []
                    for k in range(4):
                        es.append(ring[s0 + q + k]); yield   # each 8-B read atomic on its own
                    if not all((es[k] >> 32) == g0 + q + k + 1 for k in range(4)):
                        allok = False; break
                if allok:
                    for q in range(0, GRP, 4):
                        es = []
                        for k in range(4):
                            es.append(ring[s0 + q + k]); yield
                        m = [(es[k] >> 32) == g0 + q + k + 1 for k in range(4)]
                        for k in range(4):
                            if m[k]:
                                glob.setdefault(g0 + q + k, set()).add(es[k] & 0xFFFFFFFF)
                        yield
                        for k in range(4):
                            if m[k] and ring[s0 + q + k] == es[k]:
                                ring[s0 + q + k] = 0
                            yield
                    return
                yield
    pending = [writer(t) for t in targets]
    active = []
    while pending or active:
        while pending and len(active) < n_workers:
            active.append(pending.pop(0))
        w = rnd.choice(active)
        try:
            next(w)
        except StopIteration:
            active.remove(w)
    for s in range(R):   # final flush
        e = ring[s]
        if e:
            glob.setdefault((e >> 32) - 1, set()).add(e & 0xFFFFFFFF)
    # every position 0..lc-1 must hold exactly one value; values = all targets
    assert lc == n_items
    for p in range(lc):
        vals = glob.get(p)
        assert vals and len(vals) == 1, (seed, p, vals)
    got = sorted(next(iter(glob[p])) for p in range(lc))
    assert got == targets, seed


@pytest.mark.parametrize("block", range(5))
def test_every_staged_position_reaches_its_slice(block):
    for seed in range(block * 100, block * 100 + 100):
        r = random.Random(seed)
        run(seed, n_items=r.randint(1, 300), n_workers=r.randint(1, 64))
