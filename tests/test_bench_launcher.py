"""bench.py --gpus N: N ranks or a non-zero exit (CPU; nothing here touches a GPU).

The reference times one device between two synchronisations
(test_lanczos.cu:239-248); the multi-GPU line is this build's own.  The driver
may call `python bench.py --gpus 8` without torch.distributed.run: the script
must then start the 8 ranks itself, never report a 1-rank run as 8 GPUs.
"""
import io
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_world_plan():
    assert bench.world_plan(1, {}) == "run"
    assert bench.world_plan(8, {}) == "launch"
    assert bench.world_plan(2, {"WORLD_SIZE": ""}) == "launch"
    assert bench.world_plan(4, {"WORLD_SIZE": "4"}) == "run"
    assert bench.world_plan(1, {"WORLD_SIZE": "1"}) == "run"
    for gpus, w in ((1, "2"), (8, "1"), (2, "4")):
        with pytest.raises(SystemExit) as e:
            bench.world_plan(gpus, {"WORLD_SIZE": w})
        assert e.value.code != 0
    with pytest.raises(SystemExit):
        bench.world_plan(0, {})


def test_launch_cmd():
    argv = ["--gpus", "8", "--config", "c4", "--steps", "5"]
    cmd = bench.launch_cmd(argv, 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd and "--master-port=29511" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1] == os.path.join(ROOT, "bench.py")
    assert cmd[-len(argv):] == argv  # the ranks see the same --gpus N, and WORLD_SIZE = N from the launcher


def test_free_port():
    p = bench.free_port()
    assert 0 < p < 65536


def test_relay_copies_stdout_and_status():
    out = io.StringIO()
    rc = bench.relay([sys.executable, "-c", "import sys; print('{\"value\": 1}'); sys.exit(3)"], out)
    assert rc == 3
    assert out.getvalue() == '{"value": 1}\n'


def _bench(args, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, env=env, timeout=120)


@pytest.mark.parametrize("gpus,world", [(1, "2"), (8, "2"), (2, "1")])
def test_mismatch_exits_nonzero(gpus, world):
    """WORLD_SIZE disagreeing with --gpus: non-zero exit before any GPU call, no line."""
    p = _bench(["--gpus", str(gpus)], {"WORLD_SIZE": world, "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert p.stdout.strip() == ""
    assert "WORLD_SIZE" in p.stderr


def test_c4rank_needs_one_gpu():
    p = _bench(["--gpus", "2", "--config", "c4rank"], {"WORLD_SIZE": ""})
    assert p.returncode != 0 and p.stdout.strip() == ""
