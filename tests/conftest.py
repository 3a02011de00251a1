import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uigc-akka_amd", "workload", "oracle", "tests"):
    p = os.path.join(REPO, sub)
    if p not in sys.path:
        sys.path.insert(0, p)

# The tests drive the A/B variants and test hooks (CRGC_ALPHA, CRGC_XBITS, ...),
# which the library reads only under this gate (crgc_api.hip Knobs); with no
# hook variable set, every default is the production one.
os.environ["CRGC_TEST_HOOKS"] = "1"
# Slot reuse purges the swept slots after every sweep in the suite (the
# library batches them, CRGC_SLOT_REUSE_DIV=16), so every unsharded parity test
# runs its reused slots through the next merges.
os.environ.setdefault("CRGC_SLOT_REUSE_DIV", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running parity case")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def hip_mod():
    """The HIP product path.  Fails loudly if the extension or GPU is missing."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test collected on a host without a GPU")
    import crgc_hip
    crgc_hip.abi.load_library()
    return crgc_hip
