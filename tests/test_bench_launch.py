"""bench.py's launch contract on CPU: `--gpus N` outside a torchrun environment re-runs the script
under torch.distributed.run (N processes, 127.0.0.1 rendezvous) before anything touches a GPU, and
the defaults are N = 1 with a short K / W (the driver's no-flag run)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_defaults(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.gpus == 1 and a.steps > 0 and a.warmup >= 0 and a.points_per_gpu == 1e9 and a.res == 9


def test_relaunch_command(monkeypatch):
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 0

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.relaunch(bench.parse()) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_main_relaunches_before_gpu(monkeypatch):
    """main() with --gpus 2 and no WORLD_SIZE exits through relaunch without importing torch.cuda work"""
    calls = []
    monkeypatch.setattr(bench, "relaunch", lambda a: calls.append(a.gpus) or 7)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7 and calls == [2]
