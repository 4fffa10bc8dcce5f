"""bench.py --gpus N: the launch decision is made before any GPU call.

A bare `python bench.py --gpus N` (N > 1) starts its N ranks as a child
`python -m torch.distributed.run`; under a launcher WORLD_SIZE must equal --gpus or the
bench exits 2 without touching the GPU.  CPU only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_one_gpu_runs_in_process():
    assert bench.launch_plan(1, {}) == ("run", None)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == ("run", None)


def test_n_gpus_without_launcher_spawns_n_ranks():
    how, cmd = bench.launch_plan(8, {}, argv=["--gpus", "8", "--steps", "5"], port=29555)
    assert how == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    j = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[j + 1:] == ["--gpus", "8", "--steps", "5"]


def test_launcher_world_must_match():
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}) == ("run", None)
    how, msg = bench.launch_plan(4, {"WORLD_SIZE": "2"})
    assert how == "refuse" and "WORLD_SIZE=2" in msg and "--gpus 4" in msg
    how, msg = bench.launch_plan(1, {"WORLD_SIZE": "8"})
    assert how == "refuse"
    assert bench.launch_plan(0, {})[0] == "refuse"


@pytest.mark.parametrize("env_world,gpus", [("2", 4), ("8", 1)])
def test_mismatched_launch_exits_2_before_the_gpu(env_world, gpus):
    env = dict(os.environ, WORLD_SIZE=env_world, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus)],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "must equal --gpus" in r.stderr
    assert r.stdout.strip() == ""          # no bench line from a refused launch
