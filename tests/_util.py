import ctypes

import numpy as np


def cp(a: np.ndarray):
    """ctypes pointer to a contiguous numpy array."""
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def c_fps(coracle, xyz: np.ndarray, start: int, npoint: int) -> np.ndarray:
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    out = np.zeros(npoint, dtype=np.int64)
    coracle.oc_fps(cp(xyz), xyz.shape[0], int(start), int(npoint), cp(out))
    return out


def c_ball_query(coracle, pc1: np.ndarray, pc2: np.ndarray, r: float):
    pc1 = np.ascontiguousarray(pc1, dtype=np.float64)
    pc2 = np.ascontiguousarray(pc2, dtype=np.float64)
    cap = pc1.shape[0] * pc2.shape[0]
    cap = min(cap, 1 << 24)
    pairs = np.zeros((cap, 2), dtype=np.int64)
    o12 = np.zeros(pc1.shape[0], dtype=np.int8)
    o21 = np.zeros(pc2.shape[0], dtype=np.int8)
    n = coracle.oc_ball_query(cp(pc1), pc1.shape[0], cp(pc2), pc2.shape[0], float(r), cp(pairs), cap, cp(o12), cp(o21))
    return pairs[:n], o12, o21


def boundary_cloud(rng, n1: int, n2: int, r: float, scale: float = 8.0, offset=(0.0, 0.0, 110.0)):
    """Two clouds with many pairs at distance ~r (some exactly r up to rounding)."""
    off = np.asarray(offset)
    pc1 = rng.uniform(-scale, scale, size=(n1, 3)) + off
    pick = rng.integers(0, n1, size=n2)
    u = rng.normal(size=(n2, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    jitter = rng.choice([0.0, 1e-15, -1e-15, 1e-9, -1e-9, 0.3, -0.3], size=(n2, 1))
    pc2 = pc1[pick] + u * (r * (1.0 + jitter))
    half = n2 // 2
    pc2[:half] = rng.uniform(-scale, scale, size=(half, 3)) + off
    return pc1, pc2
