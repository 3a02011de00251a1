"""E12 on the oracle: Java int wraparound of recvCount and outgoing counts."""
import pytest

import wrap_streams


@pytest.mark.parametrize("name", sorted(wrap_streams.streams()))
def test_oracle_wraps_like_java_int(oracle_mod, name):
    steps, er, ee = wrap_streams.streams()[name]
    o = oracle_mod.OracleGraph()
    wrap_streams.apply(o, steps)
    wrap_streams.check(o.export(), er, ee)
    o.trace(True)
