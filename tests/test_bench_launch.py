"""bench.py's launcher logic (`--gpus N` with and without torch.distributed.run),
decided and exercised without a GPU: the rank-count / device-count checks, the
per-rank environments of the self-spawn, and a real spawn whose ranks refuse a
mismatched --gpus (the children exit before any device work)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_single_gpu_default():
    p = bench.launch_plan(None, {}, 1, "nccl")
    assert p["mode"] == "single" and p["world"] == 1 and p["envs"] == []
    assert bench.launch_plan(1, {}, 8, "nccl")["mode"] == "single"


def test_no_gpu_is_an_error():
    assert "error" in bench.launch_plan(None, {}, 0, "nccl")


def test_spawn_envs_one_rank_per_gpu():
    p = bench.launch_plan(4, {"PATH": "/x"}, 8, "nccl")
    assert p["mode"] == "spawn" and p["world"] == 4 and len(p["envs"]) == 4
    ports = {e["MASTER_PORT"] for e in p["envs"]}
    assert len(ports) == 1
    for r, e in enumerate(p["envs"]):
        assert e["RANK"] == str(r) and e["LOCAL_RANK"] == str(r) and e["WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["PATH"] == "/x"


def test_nccl_needs_a_gpu_per_rank():
    p = bench.launch_plan(2, {}, 1, "nccl")
    assert "error" in p and "2 GPUs" in p["error"]
    # under torchrun as well
    p = bench.launch_plan(None, {"WORLD_SIZE": "8"}, 4, "nccl")
    assert "error" in p
    # gloo rehearses N > 1 on one GPU
    assert bench.launch_plan(2, {}, 1, "gloo")["mode"] == "spawn"


def test_launcher_world_must_match_gpus():
    env = {"WORLD_SIZE": "4", "RANK": "1"}
    assert bench.launch_plan(4, env, 8, "nccl")["mode"] == "rank"
    assert bench.launch_plan(None, env, 8, "nccl")["world"] == 4
    p = bench.launch_plan(2, env, 8, "nccl")
    assert "error" in p and "WORLD_SIZE=4" in p["error"]
    assert "error" in bench.launch_plan(None, {"WORLD_SIZE": "x"}, 8, "nccl")
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, 1, "nccl")["mode"] == "single"


def test_bad_gpu_count():
    assert "error" in bench.launch_plan(0, {}, 8, "nccl")
    assert "error" in bench.launch_plan(-2, {}, 8, "nccl")


def test_spawned_ranks_report_failure():
    """A real self-spawn of 2 ranks whose --gpus (3) does not match the world
    they were started in (2): each child refuses before touching a device,
    and the parent returns the failing code."""
    plan = bench.launch_plan(2, dict(os.environ), 2, "gloo")
    assert plan["mode"] == "spawn"
    rc = bench.spawn_ranks(plan["envs"], ["--gpus", "3", "--dist-backend", "gloo"])
    assert rc == 2


def test_cli_refuses_nccl_without_gpus():
    """`python bench.py --gpus 2` on a host with fewer GPUs than ranks exits
    non-zero with a message, spawning nothing (no GPU here: 0 visible)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "need 2 GPUs" in r.stderr and r.stdout == ""
