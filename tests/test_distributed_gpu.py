"""GPU: the multi-rank training path on HIP tensors (two ranks sharing cuda:0 over gloo, as
bench.py's PK_BENCH_BACKEND rehearsal): TrainStep's flat-gradient all-reduce (every .grad a
view of one buffer, one collective) gives the cross-rank mean, and a real training step
leaves every rank with identical parameters (DDP semantics)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch(worker, marker):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", worker)]
    r = subprocess.run(cmd, env=dict(os.environ), cwd=ROOT, capture_output=True, text=True, timeout=220)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert marker in r.stdout


@pytest.mark.timeout(240)
def test_two_rank_flat_allreduce_on_gpu():
    """flat all-reduce mean; eager, GraphedTrainStep and PipelinedTrainer steps (graph A |
    eager all-reduce | graph B): the averaged gradient equals the mean of the ranks' own
    gradients and parameters stay identical across ranks over several replays."""
    _launch("_dist_gpu_worker.py", "dist-gpu ok")


@pytest.mark.timeout(240)
def test_sharded_inference_equals_single_rank():
    """configs[3] sharding: 2 ranks x 2 crops give bit-identical poses, IR, correspondence
    counts, metrics and C to one process over the 4 crops."""
    _launch("_dist_infer_worker.py", "sharded-infer ok")


@pytest.mark.timeout(240)
def test_rccl_flat_allreduce_world1():
    """RCCL (backend "nccl") initialised and used by the training step's gradient collective,
    world size 1 (one GPU per rank; see tests/_rccl_worker.py)."""
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_rccl_worker.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=220)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "rccl ok" in r.stdout
