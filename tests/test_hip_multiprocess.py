"""The sharded protocol between processes: G ranks, each a separate process
holding one shard on the test box's MI355X, exchanging through the product's
host transport over torch.distributed gloo (tests/mp_shard_worker.py) — the
host code of the one-process-per-GPU path (routed merges, home-slot
resolution, mark rounds, the sharded sweep) with a host collective in place of
RCCL, which refuses two ranks on one GPU.  Bit-exact against the unsharded
oracle on every trace (the multi-process path was only modelled in
Python on CPU)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return str(s.getsockname()[1])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world_size", [2, 3])
def test_shards_in_separate_processes_match_oracle(hip_mod, tmp_path, world_size):
    out = str(tmp_path / "mp.json")
    port = _port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mp_shard_worker.py"), str(r),
                               str(world_size), port, out], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world_size)]
    logs = []
    for p in procs:
        try:
            so, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(so)
    assert all(p.returncode == 0 for p in procs), "\n".join(l[-3000:] for l in logs)
    res = json.load(open(out))
    assert res["checks"] and res["identical"], res["checks"]
    assert max(c["rounds"] for c in res["checks"]) >= 2  # marks crossed processes
