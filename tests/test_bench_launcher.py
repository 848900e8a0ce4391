"""bench.py's multi-GPU entry (no GPU needed): ``python bench.py --gpus N``
outside a launcher starts N ranks under torch.distributed.run as a child
process and relays its exit code; under a launcher, WORLD_SIZE must equal
--gpus."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launcher_command():
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "3"], 8, 29511)
    assert cmd == [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   "--nproc-per-node=8", "--master-addr", "127.0.0.1", "--master-port", "29511",
                   os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3"]


def test_gpus_gt1_relays_a_child_launcher(monkeypatch):
    seen = {}

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return subprocess.CompletedProcess(cmd, 3)

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "4"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 3                       # the child's return code
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=2" in cmd and cmd[-4:] == ["--gpus", "2", "--steps", "4"]
    assert seen["env"]["MASTER_ADDR"] == "127.0.0.1"
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert "WORLD_SIZE=4" in str(ex.value.code)
