"""A torch-free process (what a JVM binding is) that merges and traces exits
cleanly: nothing in the library or its Python mirror pulls torch in behind the
caller's back (importing torch after the library has initialised the HIP
runtime made such a process abort in its exit handlers)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys
sys.path[:0] = [{pkg!r}, {tests!r}, {wl!r}]
import crgc_hip, kats
w = kats.RandomWorld(seed=7, max_actors=300, wake_every=13)
h = crgc_hip.ShadowGraph()
for b in w.steps():
    h.merge_entries(b)
    w.kill(h.trace(True).kill_set())
h.close()
assert "torch" not in sys.modules
print("ok")
"""


def test_torch_free_process_exits_cleanly():
    code = SCRIPT.format(pkg=os.path.join(REPO, "uigc-akka_amd"), tests=os.path.join(REPO, "tests"),
                         wl=os.path.join(REPO, "workload"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.returncode, p.stdout[-500:], p.stderr[-2000:])
    assert p.stdout.strip().endswith("ok")
