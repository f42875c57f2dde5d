"""bench.py's process launch (CPU only, no GPU work: --dry-run exits before anything touches
the device).  `--gpus N` without a launcher starts N rank processes itself, each with its own
RANK / LOCAL_RANK and one shared 127.0.0.1 rendezvous; under a launcher (WORLD_SIZE set) a
world size that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    e.update(kw)
    return e


def test_gpus_n_starts_n_ranks():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run"], env=_env(), capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert sorted(r["rank"] for r in lines) == [0, 1, 2, 3]
    assert all(r["world"] == 4 and r["local_rank"] == r["rank"] for r in lines)
    assert len({r["master"] for r in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")
    assert len({r["pid"] for r in lines}) == 4


def test_one_gpu_runs_in_process_and_world_mismatch_is_refused():
    out = subprocess.run([sys.executable, BENCH, "--dry-run"], env=_env(), capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0
    r = json.loads(out.stdout.strip())
    assert r["world"] == 1 and r["rank"] == 0
    bad = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dry-run"], env=_env(WORLD_SIZE="2", RANK="0"),
                         capture_output=True, text=True, timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE=2" in bad.stderr
    ok = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"],
                        env=_env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1"), capture_output=True, text=True,
                        timeout=120)
    assert ok.returncode == 0 and json.loads(ok.stdout.strip())["rank"] == 1  # under a launcher: no re-spawn


def test_failed_rank_fails_the_launch():
    """A rank that dies makes the parent exit non-zero (the others are stopped)."""
    import time
    t0 = time.time()
    out = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-run", "--dry-run-fail-rank", "1"], env=_env(),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 3
    assert time.time() - t0 < 30  # ranks 0 and 2 (sleeping) were stopped, not waited for


def test_hung_collective_times_out():
    """A rank that never joins a collective: the others' all-reduce gives up at --dist-timeout
    (the process group's timeout), exits non-zero, and the launcher stops the hung rank -- the
    run ends in seconds instead of blocking until an outer limit kills it."""
    import time
    t0 = time.time()
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--dry-run-hang-rank", "1",
                          "--dist-timeout", "5"], env=_env(), capture_output=True, text=True, timeout=170)
    assert out.returncode != 0
    assert time.time() - t0 < 90, time.time() - t0
    ok = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--dry-run-hang-rank", "5",
                         "--dist-timeout", "30"], env=_env(), capture_output=True, text=True, timeout=170)
    assert ok.returncode == 0, ok.stderr[-2000:]  # no hung rank: the collective completes


def test_plan_lanes_per_rank_shares():
    """The lane x step plans of the 40 000-sample rollout per rank: lane counts that are
    multiples of 1024 in [4096, max_lanes] covering the share, and the shapes the GPU share tests
    pin (8192 x 5, 7168 x 3, 5120 x 2, 5120 x 1 at N = 1 / 2 / 4 / 8)."""
    import math
    sys.path.insert(0, ROOT)
    import bench
    expect = {1: (8192, 5), 2: (7168, 3), 4: (5120, 2), 8: (5120, 1)}
    for n, plan in expect.items():
        share = math.ceil(40000 / n)
        assert bench.plan_lanes(share, 8192) == plan
    for share in (1, 999, 4096, 5000, 12345, 40000, 65536, 100000):
        for cap in (4096, 8192, 16384, 40960):
            L, T = bench.plan_lanes(share, cap)
            assert L % 1024 == 0 and 4096 <= L <= max(cap, 4096) and L * T >= share
    assert bench.plan_lanes(40000, 8192, lanes=4096) == (4096, 10)  # configs[1]'s 4096 envs
