"""bench.py's own N-rank launcher (no torchrun around it), on the CPU.

The driver may run ``python3 bench.py --gpus N`` without a launcher; the
parent then starts N ranks itself (``bench.launch_ranks``).  These tests run
the launcher over a small stand-in rank script: the environment each rank
sees, rank 0's stdout as the only output, a failing rank stopping the job
with its exit code, and a hang ending at the timeout.  The last test drives
the real bench.py with --gpus 2 on this GPU-less host: both ranks fail at
their first GPU call and the parent exits non-zero without a JSON line.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap
import time
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    mode = sys.argv[1]
    r = int(os.environ["RANK"])
    env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                          "MASTER_ADDR", "MASTER_PORT")}
    print("[Gloo] Rank", r, "is connected", flush=True)  # a backend's note on stdout: not the line
    print(json.dumps(env), flush=True)          # every rank prints; only rank 0's may reach the parent
    print("rank", r, "stderr", file=sys.stderr, flush=True)
    if mode == "fail" and r == 1:
        sys.exit(3)
    if mode in ("fail", "hang") and r != 1 or mode == "hang":
        time.sleep(120)                          # a rank that waits for its peers (a collective)
""")


@pytest.fixture()
def rank_script(tmp_path):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    return p


def run_launcher(tmp_path, script, mode, n, timeout):
    driver = tmp_path / "drive.py"
    driver.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {str(ROOT)!r})
        import bench
        sys.exit(bench.launch_ranks({n}, [sys.executable, {str(script)!r}, {mode!r}], {timeout}))
    """))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t = time.monotonic()
    p = subprocess.run([sys.executable, str(driver)], capture_output=True, text=True, env=env, timeout=90)
    return p, time.monotonic() - t


def test_every_rank_gets_its_environment_and_only_rank0_prints(tmp_path, rank_script):
    p, _ = run_launcher(tmp_path, rank_script, "ok", 4, 60)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1  # rank 0's stdout only
    env = json.loads(lines[0])
    assert env["RANK"] == "0" and env["LOCAL_RANK"] == "0"
    assert env["WORLD_SIZE"] == "4" and env["LOCAL_WORLD_SIZE"] == "4"
    assert env["MASTER_ADDR"] == "127.0.0.1" and 0 < int(env["MASTER_PORT"]) < 65536
    for r in range(4):  # every rank ran (stderr passes through)
        assert f"rank {r} stderr" in p.stderr
    assert "[Gloo] Rank 0 is connected" in p.stderr  # rank 0's other stdout lines go to stderr


def test_a_failing_rank_stops_the_job_with_its_code(tmp_path, rank_script):
    p, dt = run_launcher(tmp_path, rank_script, "fail", 3, 60)
    assert p.returncode == 3
    assert "rank 1 exited with 3" in p.stderr
    assert dt < 30  # the other ranks (sleeping 120 s) were killed, not waited for


def test_a_hung_job_is_killed_at_the_timeout(tmp_path, rank_script):
    p, dt = run_launcher(tmp_path, rank_script, "hang", 2, 2)
    assert p.returncode == 124
    assert "still running" in p.stderr
    assert dt < 30


def test_free_port_is_bindable():
    import socket
    port = bench.free_port()
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", port))


def test_bench_self_launches_and_fails_loudly_without_a_gpu():
    """The real bench.py, --gpus 2, no torchrun: two ranks start, both fail at
    their first GPU call on this host, the parent exits non-zero and prints
    no JSON line (a silent N=1 fallback would print one)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU host: the failure path needs a GPU-less host")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--launch-timeout", "120"], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0
    assert "exited with" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("argv,env_world,want", [
    (["--gpus", "1"], None, 1_000_000),                          # config 2
    (["--gpus", "8"], None, bench.CONFIG3_READS_PER_GPU),        # config 3: 100M reads over 8 GPUs
    (["--gpus", "2"], "2", bench.CONFIG3_READS_PER_GPU),
    (["--gpus", "1"], "4", bench.CONFIG3_READS_PER_GPU),         # torchrun's WORLD_SIZE wins
    (["--gpus", "8", "--workload", "genus"], None, 1_000_000),
    (["--gpus", "8", "--reads", "5000"], None, 5000),
])
def test_reads_default_follows_world_size(monkeypatch, argv, env_world, want):
    """N > 1 species runs default to config 3's per-GPU share (BASELINE.json configs[2])."""
    if env_world is None:
        monkeypatch.delenv("WORLD_SIZE", raising=False)
    else:
        monkeypatch.setenv("WORLD_SIZE", env_world)
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    assert bench.parse().reads == want
    assert bench.CONFIG3_READS_PER_GPU * 8 == 100_000_000


def test_block_checksum_sees_moved_and_changed_cells():
    """The multigenus exchange check: equal blocks give equal sums; a changed
    cell, swapped cells or a shifted block origin do not."""
    import torch
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.integers(0, 131, (300, 40)).astype(np.int32))
    base = bench._checksum(x, 1000)
    assert base == bench._checksum(x.to(torch.uint8), 1000)      # the narrow wire type carries the same sum
    y = x.clone()
    y[7, 3] += 1
    assert bench._checksum(y, 1000) != base
    z = x.clone()
    z[[7, 8]] = z[[8, 7]]
    if not torch.equal(z, x):
        assert bench._checksum(z, 1000) != base
    assert bench._checksum(x, 999) != base
