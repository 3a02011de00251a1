"""bench.py's own multi-rank launcher on the CPU (gloo): `--gpus N` with no
launcher around it starts N ranks through torch.distributed.run, each checks
its world size, and rank 0 reports the max-over-ranks wall time (--dry-run:
the same rendezvous, barriers and reductions, no GPU work)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=300, cwd=REPO, env=e)


def test_bench_starts_its_own_ranks():
    p = _run(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout              # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2 and out["ranks_reported"] == 2 and out["dry_run"]
    assert out["steps"] == 3 and out["ms_per_step"] > 0


def test_bench_refuses_a_world_size_other_than_gpus():
    p = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "world size 1 != --gpus 2" in p.stderr


def _dry(args):
    p = _run(args + ["--dry-run", "--steps", "1", "--warmup", "0"])
    assert p.returncode == 0, p.stderr[-2000:]
    return [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")][0]


def test_default_curve_is_one_workload():
    """The driver's --gpus 1/2/4/8 lines quote one workload: C2 per rank (at
    N > 1 the ranks' nodes as one hash-sharded graph), weak scaling, and the
    config block differs only in `parallelism`."""
    one, eight = _dry(["--gpus", "1"]), _dry(["--gpus", "8"])
    assert one["scaling"] == eight["scaling"] == "weak"
    assert one["config"]["workload"].startswith("C2")
    assert {k: v for k, v in one["config"].items() if k != "parallelism"} == \
        {k: v for k, v in eight["config"].items() if k != "parallelism"}
    assert eight["config"]["parallelism"].startswith("hash-sharded x8")


def test_c4_curve_config_is_the_same_at_every_n():
    """--workload c4: one 1e8-actor / 1e9-edge graph at every N (strong
    scaling), every producer on exactly one rank, one config block."""
    one, eight = _dry(["--gpus", "1", "--workload", "c4"]), _dry(["--gpus", "8", "--workload", "c4"])
    for out in (one, eight):
        assert out["config"]["edges"] == 1_000_000_000 and out["config"]["actors"] == 100_000_000
        assert out["config"]["workload"].startswith("C4") and out["scaling"] == "strong"
    assert one["config"]["workload"] == eight["config"]["workload"]
    assert sorted(k for ks in eight["producers"] for k in ks) == list(range(8))
