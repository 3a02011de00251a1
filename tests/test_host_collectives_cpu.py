"""crgc_transport_host's Python callbacks (crgc_hip.HostCollectives over
torch.distributed gloo) between processes on the CPU: all-gather and
all-to-all-v with gaps and uneven sizes, called through the function pointers
the library calls (tests/mp_coll_worker.py); the multi-process GPU test
(tests/test_hip_multiprocess.py) runs the whole protocol over them."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("world_size", [2, 3])
def test_host_collectives_between_processes(world_size):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "mp_coll_worker.py"), str(r), str(world_size),
                               port], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world_size)]
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-2000:] for o in outs)
    assert all(f"ok {r}" in o for r, o in enumerate(outs))
