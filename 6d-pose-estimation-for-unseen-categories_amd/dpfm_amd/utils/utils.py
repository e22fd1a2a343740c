"""Label and metric helpers of the reference utils/utils.py on the device.

C_from_sparse_P (utils/utils.py:67-79) and compute_inlier_ratio (:81-105) keep their
signatures; the batched variants used by the training step take packed pair lists.
"""
from __future__ import annotations

import torch
import yaml

from .. import ops

__all__ = ["C_from_sparse_P", "compute_inlier_ratio", "yaml_read", "C_from_sparse_P_batched",
           "inlier_ratio_batched"]


def yaml_read(path):
    with open(path, "r") as f:
        return yaml.safe_load(f)


def C_from_sparse_P(P, evecs1, evecs2):
    """Best fmap for the correspondences P [n, 2] (CAD idx, PC idx): least squares
    evecs2[P1] X = evecs1[P0] (evecs sliced to the fmap size by the caller, as at
    train.py:101). fp64 normal equations on the device (pk_cgt_lstsq)."""
    k = evecs1.shape[-1]
    if k != 30 or evecs2.shape[-1] != 30:
        raise ValueError("C_from_sparse_P kernel is built for n_fmap = 30")
    dev = evecs1.device
    P = P.to(device=dev, dtype=torch.int64).contiguous()
    n = torch.tensor([P.shape[0]], dtype=torch.int64, device=dev)
    return ops.cgt_lstsq(P[None], n, evecs1[None].float(), evecs2[None].float())[0]


def C_from_sparse_P_batched(pairs, npairs, evecs1, evecs2):
    """pairs int64 [B, cap, 2], npairs int64 [B]; evecs [B, V, >=30] -> C_gt [B, 30, 30]."""
    return ops.cgt_lstsq(pairs, npairs, evecs1, evecs2)


def compute_inlier_ratio(pred_corr, CAD, PC_aligned, threshold):
    """Fraction of correspondences closer than `threshold` under the GT alignment
    (utils/utils.py:81-105): 0-d f32 tensor, or the int 0 without correspondences."""
    total_corr = len(pred_corr)
    if total_corr == 0:
        return 0
    dev = CAD.device
    pairs = pred_corr.to(device=dev, dtype=torch.int64).contiguous()[None]
    n = torch.tensor([total_corr], dtype=torch.int32, device=dev)
    thr = torch.tensor([float(threshold)], dtype=torch.float32, device=dev)
    return ops.inlier_ratio(pairs, n, CAD.float()[None], PC_aligned.float().to(dev)[None], thr, layout=0)[0]


def inlier_ratio_batched(p_pred, npred, CAD, PC_aligned, thr):
    """p_pred int64 [B, 2, L] (row 0 CAD idx, row 1 PC idx) -> IR f32 [B]."""
    return ops.inlier_ratio(p_pred, npred, CAD, PC_aligned, thr, layout=1)
