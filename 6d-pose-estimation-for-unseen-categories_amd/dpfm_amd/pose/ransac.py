"""RANSAC + Umeyama pose fit — drop-in for scripts/test_RANSAC.py:288-310
`ransac_registration` (Open3D registration_ransac_based_on_correspondence with
TransformationEstimationPointToPoint(False), ransac_n = 4,
RANSACConvergenceCriteria(4000000, ...) whose confidence clamps to 1 so every
iteration runs). The hypotheses run on the device (pk_ransac); the drawn index sets
come from the documented splitmix64 hash of `seed` (Open3D's own RNG is not
reproducible), or are passed explicitly."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .. import ops


@dataclass
class RegistrationResult:
    """The fields of open3d.pipelines.registration.RegistrationResult the reference reads."""
    transformation: np.ndarray
    fitness: float
    inlier_rmse: float
    best_hypothesis: int


def _as_tensor(x, dtype, device):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=device).contiguous()


def ransac_registration(cad_xyz, pc_xyz, P, distance_threshold=0.05, num_iterations=80000,
                        max_iteration: int = 4000000, seed: int = 0, hypotheses=None, device=None):
    """cad_xyz [V1,3], pc_xyz [V2,3] (numpy or tensors), P [n,2] (CAD idx, PC idx).
    `num_iterations` is the reference's confidence argument (clamped to 1: no early exit).
    Returns a RegistrationResult whose `.transformation` is the 4x4 f64 pose."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    src = _as_tensor(cad_xyz, torch.float64, dev)
    dst = _as_tensor(pc_xyz, torch.float64, dev)
    cor = _as_tensor(np.asarray(P).reshape(-1, 2), torch.int32, dev)
    n = cor.shape[0]
    so = torch.tensor([0, src.shape[0]], dtype=torch.int64, device=dev)
    do = torch.tensor([0, dst.shape[0]], dtype=torch.int64, device=dev)
    co = torch.tensor([0, n], dtype=torch.int64, device=dev)
    hyps = hoff = None
    H = int(max_iteration)
    if hypotheses is not None:
        hyps = _as_tensor(hypotheses, torch.int32, dev)
        H = hyps.shape[0]
        hoff = torch.tensor([0, H], dtype=torch.int64, device=dev)
    T, st = ops.ransac(src, so, dst, do, cor, co, H, seed=seed, max_dist=distance_threshold, hyps=hyps, hyp_off=hoff)
    st = st[0].cpu().numpy()
    return RegistrationResult(T[0].cpu().numpy(), float(st[0]), float(st[1]), int(st[2]))


def ransac_batched(src, src_off, dst, dst_off, corres, cor_off, H: int, seed: int = 0, max_dist: float = 0.05):
    """All crops at once (device tensors, packed layout): (T f64 [B,4,4], stats f64 [B,3])."""
    return ops.ransac(src, src_off, dst, dst_off, corres, cor_off, H, seed=seed, max_dist=max_dist)
