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


def test_gpus2_reductions_report_slowest_rank():
    """at N > 1 the roofline is the SLOWEST rank's (as `value` is) and
    the line carries the per-rank spread.  Two gloo ranks on the CPU with synthetic
    launch times (rank r: (1 + r / 10) ms) through bench.py's own reduction and
    roofline code (RPCCRC_BENCH_REDUCE_ONLY)."""
    env = dict(os.environ, RPCCRC_BENCH_REDUCE_ONLY="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    r = lines[0]["roofline"]
    assert r["per_rank"]["ranks"] == 2
    assert r["per_rank"]["min_us"] == 1000.0 and r["per_rank"]["max_us"] == 1100.0
    assert r["avg_launch_us"] == 1100.0
    algo = (1 << 23) * (4096 + 4)  # C3, the N > 1 default: 8M x 4 KiB per rank
    assert r["algo_bytes_per_launch"] == algo
    assert abs(r["achieved"] - algo / 1.1e-3 / 1e9) < 0.1
    # value: both ranks' bytes over the slowest rank's wall time
    assert abs(lines[0]["value"] - 2 * (1 << 23) * 4096 / 1.1e-3 / (1 << 30)) < 0.1


def _reduce_only(extra_env):
    env = dict(os.environ, RPCCRC_BENCH_REDUCE_ONLY="1", **extra_env)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    return lines[0]


def test_gpus2_per_rank_crc_check():
    """the N > 1 line says whether every rank's CRCs were right.  Two
    gloo ranks run bench.py's own check (rank_crc_check against the reference crc.c,
    reduce_crc_check over the ranks) on a CPU-made shard each; with
    RPCCRC_BENCH_BAD_RANK=1 rank 1 reports one corrupted CRC."""
    good = _reduce_only({})
    assert good["ranks_crc_ok"] is True
    c = good["ranks_crc_check"]
    assert c["ranks"] == 2 and c["ranks_ok"] == 2 and c["mismatches"] == 0 and c["bodies_checked"] == 128
    bad = _reduce_only({"RPCCRC_BENCH_BAD_RANK": "1"})
    assert bad["ranks_crc_ok"] is False
    c = bad["ranks_crc_check"]
    assert c["ranks_ok"] == 1 and c["mismatches"] == 1 and c["bodies_checked"] == 128


def test_live_traffic_launch_selection():
    """bench.py's live-traffic reading (pick_launch_traffic): the big launches are
    chosen on FETCH_SIZE and the same launch positions are read from WRITE_SIZE, so a
    few write outliers (dirty lines written back during one launch, r05final10) or
    the big-body route's tiny launches do not stand for the product's launches."""
    sys.path.insert(0, REPO)
    import bench

    fetch = [2097487.0, 2097463.0, 2097462.0, 2097462.0, 12.0, 2097462.0]
    write = [159499.0, 160001.0, 4185.0, 4186.0, 90.0, 4185.0]
    f, w = bench.pick_launch_traffic(fetch, write)
    assert (f, w) == (2097462.0, 4186.0)
    # an outlier on a minority of launches does not move the median
    f, w = bench.pick_launch_traffic([100.0] * 5, [9000.0, 10.0, 10.0, 10.0, 9000.0])
    assert (f, w) == (100.0, 10.0)
    # the tiny launches are left out of both
    f, w = bench.pick_launch_traffic([100.0, 1.0, 1.0, 100.0, 1.0], [10.0, 0.0, 0.0, 10.0, 0.0])
    assert (f, w) == (100.0, 10.0)
    # different launch counts between the passes: writes within half their median
    f, w = bench.pick_launch_traffic([100.0, 100.0], [10.0, 10.0, 1.0, 10.0])
    assert (f, w) == (100.0, 10.0)
