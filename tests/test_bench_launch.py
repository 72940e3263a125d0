"""bench.py's N>1 launch path on the CPU (the driver's `python bench.py
--gpus 8` exited before doing any work).  Without WORLD_SIZE, bench.py must start
torch.distributed.run itself -- as a child, before importing torch or touching a GPU
-- with one rank per GPU on a 127.0.0.1 rendezvous.  RPCCRC_BENCH_LAUNCH_ONLY makes
each rank report how it was started and stop before any device work."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(n, *extra):
    env = dict(os.environ, RPCCRC_BENCH_LAUNCH_ONLY="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "2", *extra],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, lines, p.stderr


def test_gpus2_self_launches_two_ranks():
    """N > 1 defaults to BASELINE configs[3] (C3: 8M x 4 KiB per rank, 64M over 8 GPUs)."""
    rc, lines, err = _launch(2)
    assert rc == 0, err[-3000:]
    assert sorted(x["rank"] for x in lines) == [0, 1], lines
    assert all(x["world"] == 2 and x["gpus"] == 2 and x["master"] == "127.0.0.1" for x in lines)
    assert sorted(x["local_rank"] for x in lines) == [0, 1]
    assert all(x["config"] == "c3" for x in lines), lines


def test_gpus2_explicit_config_kept():
    rc, lines, err = _launch(2, "--config", "ns")
    assert rc == 0, err[-3000:]
    assert [x["config"] for x in lines] == ["ns", "ns"], lines


def test_gpus1_runs_in_process():
    """N = 1 defaults to the north star (1M x 4 KiB), the config BASELINE's metric names."""
    rc, lines, err = _launch(1)
    assert rc == 0, err[-3000:]
    assert lines == [{"rank": 0, "world": 1, "local_rank": 0, "gpus": 1, "master": None, "config": "ns"}]
