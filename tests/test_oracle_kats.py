"""Pin the CPU oracle against the reference's own test expectations.

The reference ships no golden vectors for ShadowGraph; its integration specs
are the known answers.  Each scenario here replays one spec's message sequence
through the mutator mirror and asserts the termination outcome the spec
asserts (see tests/kats.py for the file:line of each spec).
"""
import pytest

import kats


@pytest.mark.parametrize("name", sorted(kats.SCENARIOS))
def test_oracle_scenario(oracle_mod, name):
    g = oracle_mod.OracleGraph()
    kats.run_scenario(g, kats.SCENARIOS[name]())


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_random_spec_complete_and_sound(oracle_mod, seed):
    # RandomSpec.scala: every spawned actor is eventually collected, and the
    # runner asserts no actor is stopped while it still has mail or a live
    # descendant.
    g = oracle_mod.OracleGraph()
    collected, everyone = kats.run_random(g, seed=seed, max_actors=300)
    assert collected == everyone
    assert g.live_count() == 1  # only the root remains


def test_many_messages_uses_forced_flushes(oracle_mod):
    steps = kats.many_messages()
    batches = [s[1] for s in steps if s[0] == "merge"]
    busy = sum(int((b.flags & 1).sum()) for b in batches)
    # 4*32767 sends at <=16383 per entry and receipts at <=32767 per entry
    assert busy >= (4 * 32767) // 16383 - 1
    for b in batches:
        assert b.recv_count.max(initial=0) <= 32767
