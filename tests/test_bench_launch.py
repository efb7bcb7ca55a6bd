"""bench.py's launch decision (`--gpus N` measures N ranks whoever starts it).

CPU only: the decision is made before anything touches the GPU, so it is tested here on the
function itself and on the script's refusal path (no GPU visible in this container)."""

import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


@pytest.mark.parametrize("gpus, env, ndev, plan", [
    (1, {}, 1, ("run", None)),
    (1, {}, 0, ("run", None)),                      # single rank: the run itself reports a missing GPU
    (8, {}, 8, ("spawn", 8)),                       # the driver's `python bench.py --gpus 8`
    (2, {}, 8, ("spawn", 2)),
    (8, {"WORLD_SIZE": "8"}, 8, ("run", None)),     # already under torch.distributed.run
    (2, {"CHM_DIST_BACKEND": "gloo"}, 1, ("spawn", 2)),  # gloo rehearsal: ranks share one GPU
])
def test_launch_plan(gpus, env, ndev, plan):
    assert bench.launch_plan(gpus, env, ndev) == plan


@pytest.mark.parametrize("gpus, env, ndev, match", [
    (8, {}, 1, "8 RCCL ranks"),                     # would silently time fewer GPUs
    (8, {"WORLD_SIZE": "1"}, 8, "WORLD_SIZE is 1"),
    (2, {"WORLD_SIZE": "4"}, 8, "WORLD_SIZE is 4"),
    (0, {}, 8, "at least one"),
])
def test_launch_plan_refuses(gpus, env, ndev, match):
    plan, why = bench.launch_plan(gpus, env, ndev)
    assert plan == "refuse" and match in why


def test_bench_refuses_more_ranks_than_gpus():
    """`python bench.py --gpus 2` with no launcher and no GPU exits non-zero before any rank starts
    (it would otherwise have printed n_gpus: 1)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "CHM_DIST_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "RCCL ranks" in r.stderr and "{" not in r.stdout


def test_spawn_command_line(monkeypatch):
    """The spawned launcher is torch.distributed.run on 127.0.0.1 with N processes, running this
    same script with the caller's arguments."""
    seen = {}

    class R:
        returncode = 0

    def fake_run(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    assert bench.spawn_ranks(4, ["--gpus", "4", "--steps", "3"]) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
