"""bench.py's multi-GPU launch path on CPU (gloo): `--gpus N` spawns N fresh worker
processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set per worker), each rank
owns a contiguous block of the job's windows and the decoded frames are all-gathered once at the end
(latentsync_amd/shard.py).  `--plumbing` replaces only the window compute with a
stand-in that writes each window's global index into its frames, so the gathered
clip order is checked exactly.  Also: a failing rank ends the job with a non-zero
status, and a hung rank makes the others' collective time out."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--plumbing", *args], cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _line(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_spawned_ranks_gather_in_clip_order(n):
    r = _bench("--gpus", str(n), "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr
    res = _line(r)
    assert res["n_gpus"] == n  # from the process group, not from the flag
    assert res["plumbing"]["clip_order_ok"]
    assert res["plumbing"]["gathered_windows"] == n * 3 * res["config"]["windows_per_batch"]
    assert res["plumbing"]["backend"] == ("gloo" if n > 1 else "none")
    assert res["scaling"] == "weak" and res["config"]["global_batch"] == n * res["config"]["windows_per_batch"] * 16


def test_torchrun_style_worker_env():
    """Under torchrun the process is already a worker: WORLD_SIZE must match --gpus."""
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--plumbing", "--gpus", "1"], cwd=REPO,
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_failing_rank_fails_the_job():
    r = _bench("--gpus", "2", "--steps", "2", "--fail-rank", "1", "--dist-timeout", "30")
    assert r.returncode != 0
    assert "injected failure on rank 1" in r.stderr


def test_hung_rank_times_out_the_collective():
    r = _bench("--gpus", "2", "--steps", "2", "--stall-rank", "1", "--dist-timeout", "4")
    assert r.returncode != 0
    assert "[bench rank 0] failed" in r.stderr
