"""bench.py's rank launcher (CPU): `python bench.py --gpus N` without torch.distributed.run
starts N ranks as a child job instead of silently timing one GPU; a rank whose WORLD_SIZE
disagrees with --gpus refuses to run."""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launcher_cmd_spawns_n_ranks():
    b = _bench()
    argv = ["--gpus", "4", "--steps", "7", "--warmup", "2"]
    cmd = b.launcher_cmd(argv, {})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")
    assert b.launcher_cmd(["--gpus=2"], {})[4] == "--nproc-per-node=2"


@pytest.mark.parametrize("argv,env", [(["--gpus", "1"], {}), ([], {}),
                                      (["--gpus", "8"], {"WORLD_SIZE": "8", "RANK": "3"})])
def test_launcher_cmd_none_inside_a_rank_or_single_gpu(argv, env):
    assert _bench().launcher_cmd(argv, env) is None


def test_rank_world_mismatch_refuses():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)
