"""The shard exchange's error discipline on the CPU.

crgc_xpost.hpp is the posting and waiting logic RcclTransport runs
(crgc_transport.hip); tests/native/xpost_fake.cpp drives it with fake ranks:
a failing send or receive still posts every other operation, closes the group
and aborts the communicator, and a host wait on a rank whose peer failed or
hung ends with an error instead of blocking.
"""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exchange_error_paths_with_fake_ranks(tmp_path):
    exe = tmp_path / "xpost_fake"
    src = os.path.join(REPO, "tests", "native", "xpost_fake.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-pthread", src, "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "xpost ok" in r.stdout
