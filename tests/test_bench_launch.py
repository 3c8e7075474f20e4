"""bench.py --gpus N > 1 started as a plain process (the driver's 1-GPU command shape): it must
launch its N ranks itself through torch.distributed.run as a child process and exit with the
child's return code.  The child is mocked here (no GPU, no ranks)."""
import subprocess
import sys

import pytest

import bench


def test_launcher_command_shape():
    cmd = bench.launcher_cmd(["--gpus", "4", "--steps", "20", "--warmup", "5"], 4, 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29512"
    i = [k for k, a in enumerate(cmd) if a.endswith("bench.py")][0]
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "20", "--warmup", "5"]


@pytest.mark.parametrize("rc", [0, 1, 3])
def test_self_launch_propagates_return_code(rc):
    seen = []

    def fake_run(cmd):
        seen.append(cmd)
        return subprocess.CompletedProcess(cmd, rc)

    assert bench.self_launch(["--gpus", "2"], 2, run=fake_run) == rc
    assert len(seen) == 1 and "torch.distributed.run" in seen[0]


def test_main_self_launches_without_world_size(monkeypatch):
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20", "--warmup", "5"])
    monkeypatch.setattr(bench, "self_launch", lambda argv, n: calls.append((list(argv), n)) or 7)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    assert calls == [(["--gpus", "8", "--steps", "20", "--warmup", "5"], 8)]


def test_main_inside_torchrun_does_not_relaunch(monkeypatch):
    """With WORLD_SIZE set (a rank of torch.distributed.run) there is no second launch: a
    WORLD_SIZE that disagrees with --gpus is an error before anything touches the GPU."""
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    monkeypatch.setattr(bench, "self_launch", lambda argv, n: pytest.fail("relaunched inside torchrun"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE=2" in str(e.value.code)


@pytest.mark.parametrize("gpus,flag,want", [("1", [], "4"), ("2", [], "8"), ("1", ["--hw-queues", "0"], "4"),
                                            ("1", ["--hw-queues", "8"], "8"), ("2", ["--hw-queues", "16"], "16")])
def test_hw_queues_flag(monkeypatch, gpus, flag, want):
    """--hw-queues sets GPU_MAX_HW_QUEUES before anything touches HIP (default: the environment's at
    --gpus 1, 8 with more ranks; 0 keeps the environment's value, here the box's 4)."""
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setenv("WORLD_SIZE", "3")  # stops main() at the WORLD_SIZE check, before any GPU work
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", gpus] + flag)
    with pytest.raises(SystemExit):
        bench.main()
    import os
    assert os.environ["GPU_MAX_HW_QUEUES"] == want


def test_priorities_parser():
    assert bench.parse_priorities("0,-1,0") == [0, -1, 0]
    for bad in ("", "1", "0,x", "-2"):
        with pytest.raises(SystemExit):
            bench.parse_priorities(bad)
