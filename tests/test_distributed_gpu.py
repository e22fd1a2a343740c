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


@pytest.mark.timeout(240)
def test_two_rank_flat_allreduce_on_gpu():
    env = dict(os.environ)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "_dist_gpu_worker.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=220)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "dist-gpu ok" in r.stdout
