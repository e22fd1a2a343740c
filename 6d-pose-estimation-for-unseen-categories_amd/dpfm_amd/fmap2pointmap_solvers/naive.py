"""Naive fmap -> point map (reference fmap2pointmap_solvers/naive.py:6-34) on the HIP
feature-distance kernel (MFMA contraction + fused argmin; the [V1, V2] matrix is never
materialised)."""
from __future__ import annotations

import torch

from .. import ops


def _one(x: torch.Tensor) -> torch.Tensor:
    return x if x.dim() == 3 else x[None]


def nn_query(feat_x, feat_y, dim=-2):
    """argmin_i ||feat_x[i] - feat_y[j]|| for every j (naive.py:23-34); feat_x [V1, C],
    feat_y [V2, C] on the device. C <= 30 runs on the feature-distance kernel (zero columns
    appended up to its 30-wide contraction leave every distance unchanged); wider features
    take torch.cdist + argmin on the device, the reference's own formula."""
    if dim not in (-2, 0):
        raise ValueError("nn_query reduces over the first (V1) dimension")
    if feat_x.dim() != 2 or feat_y.dim() != 2 or feat_x.shape[1] != feat_y.shape[1]:
        raise ValueError("nn_query takes feat_x [V1, C] and feat_y [V2, C]")
    if not feat_x.is_cuda:
        raise ops._lib.PoseKernError("nn_query runs on HIP devices only (no CPU fallback)")
    V1, V2 = feat_x.shape[0], feat_y.shape[0]
    C = feat_x.shape[1]
    dev = feat_x.device
    if C > 30:
        return torch.cdist(feat_x.float(), feat_y.float()).argmin(dim=0)
    if C < 30:
        feat_x = torch.nn.functional.pad(feat_x.float(), (0, 30 - C))
        feat_y = torch.nn.functional.pad(feat_y.float(), (0, 30 - C))
    eye = torch.eye(30, dtype=torch.float32, device=dev)[None]
    n1 = torch.tensor([V1], dtype=torch.int32, device=dev)
    n2 = torch.tensor([V2], dtype=torch.int32, device=dev)
    idx, _ = ops.feat_dist_topk(_one(feat_x.float()), eye, _one(feat_y.float()), n1, n2, 1)
    return idx[0, :, 0]


def naive_fmap2pointmap(C12, evecs_x, evecs_y, **kwargs):
    """Convert a functional map to a point-to-point map: returns int64 [2, V2] =
    stack([p2p, arange(V2)])."""
    if C12.dim() == 3:
        C12 = C12.squeeze(0)
    V1, V2 = evecs_x.shape[0], evecs_y.shape[0]
    dev = evecs_x.device
    n1 = torch.tensor([V1], dtype=torch.int32, device=dev)
    n2 = torch.tensor([V2], dtype=torch.int32, device=dev)
    idx, _ = ops.feat_dist_topk(_one(evecs_x.float()), C12[None].float(), _one(evecs_y.float()), n1, n2, 1)
    pp = idx[0, :, 0]
    return torch.stack([pp, torch.arange(V2, device=dev, dtype=torch.int64)], 0)
