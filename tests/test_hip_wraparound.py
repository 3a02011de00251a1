"""E12 on the device: the HIP merge wraps int32 counts exactly like the oracle
(and Java) through entries, deltas and undo logs; traces agree after it."""
import pytest

import wrap_streams

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(wrap_streams.streams()))
def test_hip_wraps_like_java_int(hip_mod, oracle_mod, name):
    steps, er, ee = wrap_streams.streams()[name]
    h, o = hip_mod.ShadowGraph(), oracle_mod.OracleGraph()
    wrap_streams.apply(h, steps)
    wrap_streams.apply(o, steps)
    sh = h.export()
    assert sh == o.export()
    wrap_streams.check(sh, er, ee)
    rh, ro = h.trace(True), o.trace(True)
    assert rh.garbage_set() == ro.garbage_set() and rh.kill_set() == ro.kill_set()
    assert rh.pseudo_roots == ro.pseudo_roots and rh.n_live == ro.n_live
