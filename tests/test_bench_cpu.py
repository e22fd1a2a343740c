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


def test_train_workload_names_the_config():
    """The training line names the BASELINE.json config it measures and its true global batch:
    configs[1] on one GPU, configs[2] for 2 ranks x 16 (--gpus 2 --global-batch 32), and weak
    scaling (32 per rank) otherwise."""
    b = _bench()
    assert b.train_workload(32, 1024, 1).startswith("configs[1] shape") and "global batch 32" in b.train_workload(32, 1024, 1)
    w2 = b.train_workload(16, 1024, 2)
    assert w2.startswith("configs[2]") and "global batch 32" in w2 and "B=16" in w2
    w2w = b.train_workload(32, 1024, 2)
    assert "global batch 64" in w2w and "weak scaling" in w2w and not w2w.startswith("configs[2]")
    assert "global batch 256" in b.train_workload(32, 1024, 8)


def test_global_batch_divides_over_ranks():
    b = _bench()
    import argparse
    a = argparse.Namespace(global_batch=32, batch=32)
    b.apply_global_batch(a, 2)
    assert a.batch == 16
    a = argparse.Namespace(global_batch=None, batch=32)
    b.apply_global_batch(a, 2)
    assert a.batch == 32
    with pytest.raises(SystemExit):
        b.apply_global_batch(argparse.Namespace(global_batch=30, batch=32), 4)


def test_gloo_world2_train_config(tmp_path):
    """At world size 2 (gloo, CPU) the config dict the training line would print: configs[2] by name
    with --global-batch 32, per-rank B = 16, parallelism dp2."""
    script = tmp_path / "w.py"
    script.write_text(f"""
import importlib.util, json, os, sys
import torch.distributed as dist
spec = importlib.util.spec_from_file_location("bench_mod", {os.path.join(ROOT, "bench.py")!r})
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
dist.init_process_group("gloo")
w = dist.get_world_size()
sys.argv = ["bench.py", "--gpus", "2", "--global-batch", "32"]
a = b.parse(); b.apply_global_batch(a, w)
out = dict(workload=b.train_workload(a.batch, a.points, w), global_batch=a.batch * w, parallelism=f"dp{{w}}")
if dist.get_rank() == 0:
    print(json.dumps(out))
dist.destroy_process_group()
""")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", "29561", str(script)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][0]
    cfg = json.loads(line)
    assert cfg["workload"].startswith("configs[2]") and cfg["global_batch"] == 32 and cfg["parallelism"] == "dp2"
