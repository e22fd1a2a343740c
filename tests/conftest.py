import ctypes
import os
import subprocess
import sys

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")  # see dpfm_amd/__init__.py (HIP-graph memset replays)

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")
for p in (ROOT, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def coracle():
    """The plain-C oracle (oracle/c/oracle.c), built on demand."""
    so = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")], stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(so)
    P, I, I64, D, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double, ctypes.c_uint64
    lib.oc_fps.argtypes = [P, I, I, I, P]
    lib.oc_ball_query.argtypes = [P, I, P, I, D, P, I64, P, P]
    lib.oc_ball_query.restype = I64
    lib.oc_hyp_index.argtypes = [U64, I64, I, ctypes.c_int32]
    lib.oc_hyp_index.restype = ctypes.c_int32
    lib.oc_umeyama.argtypes = [P, P, I, P, P]
    lib.oc_ransac.argtypes = [P, P, P, I, P, U64, I64, D, P, P]
    lib.oc_icp.argtypes = [P, I, P, I, P, D, I, D, D, P, P]
    return lib


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
