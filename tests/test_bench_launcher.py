"""CPU: bench.py's own rank launcher (``python bench.py --gpus N`` without
torchrun, the driver's scaling command).  The parent process must start the N
ranks as a child torch.distributed.run -- never touching the GPU, never
re-executing itself -- and must refuse to time fewer ranks than asked."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _args(argv):
    import bench
    return bench.parse(argv)


def test_rank_command_is_a_torchrun_child_on_localhost():
    import bench
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    cmd = bench.rank_command(_args(argv), argv, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert "--master-port=29555" in cmd
    assert cmd[-len(argv) - 1] == os.path.join(REPO, "bench.py")
    assert cmd[-len(argv):] == argv        # the ranks see the same --gpus / steps / warmup


def test_launcher_refuses_fewer_devices_than_ranks():
    import bench
    calls = []
    rc = bench.launch_ranks(_args(["--gpus", "8"]), ["--gpus", "8"], device_count=1,
                            run=lambda *a, **k: calls.append(a) or 0)
    assert rc == 2 and not calls


@pytest.mark.parametrize("child_rc", [0, 1])
def test_launcher_runs_ranks_and_returns_their_status(child_rc):
    import bench
    seen = {}

    def run(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return child_rc

    argv = ["--gpus", "2", "--steps", "3"]
    rc = bench.launch_ranks(_args(argv), argv, device_count=8, run=run)
    assert rc == child_rc
    assert "--nproc-per-node=2" in seen["cmd"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"   # dmabuf IPC for RCCL
    assert "WORLD_SIZE" not in os.environ                       # the parent stays rank-less


def test_main_takes_the_launcher_path_without_world_size(monkeypatch):
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    got = {}

    def fake_launch(args, argv):
        got["gpus"], got["argv"] = args.gpus, argv
        return 0

    monkeypatch.setattr(bench, "launch_ranks", fake_launch)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and got == {"gpus": 4, "argv": ["--gpus", "4", "--steps", "2"]}


def test_main_refuses_world_size_mismatch(monkeypatch):
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 2
