"""bench.py launcher logic (CPU, nothing launched): `python bench.py --gpus N` started as a
plain process re-runs itself as N torchrun ranks in a child process (never exec), one rank
per GPU, with the driver's flags passed through (reference launch: main.py:133-154)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_launch_command_shape():
    import bench
    a = type("A", (), {"gpus": 8})()
    cmd = bench.launch_command(a, ["--gpus", "8", "--steps", "5", "--warmup", "2"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5", "--warmup", "2"]


def test_gpus_n_spawns_child_torchrun(monkeypatch):
    import bench
    calls = []

    def fake_call(cmd, env=None):
        calls.append((cmd, env))
        return 3

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 3  # the child's exit status is the bench's
    (cmd, env), = calls
    assert "--nproc-per-node=2" in cmd and cmd[-4:] == ["--gpus", "2", "--steps", "3"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_refuses_timing_switches():
    """A DVIE_*_DBG variable (timing-only kernel ablations, wrong results) makes bench.py exit
    non-zero before anything runs."""
    import bench
    with pytest.raises(SystemExit) as e:
        bench.refuse_timing_switches({"DVIE_HALO_DBG": "8"})
    assert e.value.code == 2
    bench.refuse_timing_switches({"DVIE_HALO_DBG": "", "DVIE_1X1_DBG": "0", "DVIE_PRECISION": "bf16"})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1"], capture_output=True,
                       text=True, env=dict(os.environ, DVIE_1X1_DBG="2"), timeout=120)
    assert r.returncode == 2 and "DVIE_1X1_DBG" in r.stderr
