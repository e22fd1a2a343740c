"""Pose metrics of scripts/test_RANSAC.py:77-81, 154-238 with the reference's
signatures. The per-point work (ADD, the per-row "xyz direction" distances and the
1-D nearest-neighbour ADD-S) runs in pk_pose_metrics for any number of crops."""
from __future__ import annotations

import numpy as np
import torch

from .. import ops


def _metrics(pts3d, pose_gt, pose_pred, device=None):
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    cad = torch.as_tensor(np.asarray(pts3d, dtype=np.float64), device=dev).contiguous()
    off = torch.tensor([0, cad.shape[0]], dtype=torch.int64, device=dev)
    Te = torch.as_tensor(np.asarray(pose_pred, dtype=np.float64).reshape(1, 4, 4), device=dev)
    Tg = torch.as_tensor(np.asarray(pose_gt, dtype=np.float64).reshape(1, 4, 4), device=dev)
    return ops.pose_metrics(cad, off, cad.shape[0], Te, Tg)[0].cpu().numpy()


def add(T_est, T_gt, pcd, diameter, percentage=0.1):
    """Mean distance between the model under the two poses, and whether it is below
    percentage * diameter (test_RANSAC.py:162-173)."""
    e = float(_metrics(pcd, T_gt, T_est)[0])
    return e, int(e < diameter * percentage)


def compute_add_score(pts3d, diameter, pose_gt, pose_pred, percentage=0.1):
    m = _metrics(pts3d, pose_gt, pose_pred)[1:4].astype(np.float32)
    return (m < diameter * percentage).sum() / 3


def compute_adds_score(pts3d, diameter, pose_gt, pose_pred, percentage=0.1):
    t = np.asarray(pose_pred)[:3, 3]
    m = _metrics(pts3d, pose_gt, pose_pred)[4:7].astype(np.float32)
    m[np.isnan(t)] = np.inf
    return (m < diameter * percentage).sum() / 3


def get_angular_error(R_exp, R_est):
    return abs(np.arccos(min(max(((np.matmul(R_exp.T, R_est)).trace() - 1) / 2, -1.0), 1.0)))


def pose_metrics_batched(cad, off, nmax, T_est, T_gt):
    """Device tensors: f64 [B, 7] = (ADD, xyz-direction means x3, ADD-S means x3)."""
    return ops.pose_metrics(cad, off, nmax, T_est, T_gt)
