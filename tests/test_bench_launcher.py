"""bench.py --gpus N started without a launcher starts its N ranks itself:
the children get torch.distributed.run's environment, rendezvous on 127.0.0.1, and a failing
rank makes the launcher exit non-zero and stop the others.  CPU only (gloo)."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["LOCAL_RANK"] == str(rank)
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    if "--fail" in sys.argv and rank == 1:
        sys.exit(3)
    dist.init_process_group("gloo")
    t = torch.tensor([rank + 1])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "sum": int(t.item()), "argv": sys.argv[1:]}), flush=True)
    dist.destroy_process_group()
""")


@pytest.fixture
def rank_script(tmp_path):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    return str(p)


def test_launch_two_ranks(rank_script, capfd):
    rc = bench.launch_ranks(2, argv=["--gpus", "2"], script=rank_script)
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    line = [l for l in out if l.startswith("{")]
    assert len(line) == 1, out   # rank 0 alone prints
    import json
    d = json.loads(line[0])
    assert d == {"n_gpus": 2, "sum": 3, "argv": ["--gpus", "2"]}


def test_failing_rank_fails_the_launch(rank_script):
    # rank 1 exits 3 before the rendezvous; rank 0 would wait in init_process_group, so the
    # launcher must stop it and return the failing status
    rc = bench.launch_ranks(2, argv=["--fail"], script=rank_script)
    assert rc == 3


def test_world_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
