"""Upstream DPFM helpers used by the reference (DPFM/dpfm/utils.py, un-vendored submodule,
imported at dataset/object.py:14, modeling/dpfm.py:14, utils/loss.py:3).

Same names and argument meaning as upstream; the compute runs in libposekern.so.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


def farthest_point_sample(xyz: torch.Tensor, ratio: float, start: Optional[int] = None,
                          npoint: Optional[int] = None) -> torch.Tensor:
    """xyz [3, N] (as at dataset/object.py:147) -> int64 [npoint] on xyz.device.

    npoint = int(ratio * N) like upstream. `start` defaults to torch.randint(0, N) as
    upstream draws it; pass it explicitly for reproducible (bit-exact) results.
    """
    if not xyz.is_cuda:
        raise ops._lib.PoseKernError("farthest_point_sample runs on the HIP device only")
    N = xyz.shape[1]
    if npoint is None:
        npoint = int(ratio * N)
    if start is None:
        start = int(torch.randint(0, N, (1,)).item())
    pts = xyz.t().contiguous().to(torch.float32)
    dev = xyz.device
    off = torch.tensor([0, N], dtype=torch.int64, device=dev)
    st = torch.tensor([start], dtype=torch.int32, device=dev)
    npt = torch.tensor([npoint], dtype=torch.int32, device=dev)
    return ops.fps_packed(pts, off, N, st, npt, npoint)[0]


def get_mask(evals1: torch.Tensor, evals2: torch.Tensor, gamma: float = 0.5, device=None) -> torch.Tensor:
    """Resolvent mask (upstream dpfm/utils.py::get_mask) -> [K2, K1]."""
    scaling_factor = max(torch.max(evals1), torch.max(evals2))
    evals1, evals2 = evals1 / scaling_factor, evals2 / scaling_factor
    evals_gamma1 = (evals1 ** gamma)[None, :]
    evals_gamma2 = (evals2 ** gamma)[:, None]
    M_re = evals_gamma2 / (evals_gamma2.square() + 1) - evals_gamma1 / (evals_gamma1.square() + 1)
    M_im = 1 / (evals_gamma2.square() + 1) - 1 / (evals_gamma1.square() + 1)
    return M_re.square() + M_im.square()


def get_mask_batched(evals1: torch.Tensor, evals2: torch.Tensor, gamma: float = 0.5) -> torch.Tensor:
    """get_mask for every crop at once: evals [B, K1], [B, K2] -> [B, K2, K1] (same
    arithmetic per crop; one launch sequence instead of a Python loop over crops)."""
    s = torch.maximum(evals1.max(dim=1).values, evals2.max(dim=1).values)[:, None]
    e1, e2 = evals1 / s, evals2 / s
    g1 = (e1 ** gamma)[:, None, :]
    g2 = (e2 ** gamma)[:, :, None]
    M_re = g2 / (g2.square() + 1) - g1 / (g1.square() + 1)
    M_im = 1 / (g2.square() + 1) - 1 / (g1.square() + 1)
    return M_re.square() + M_im.square()


class WeightedBCELoss(nn.Module):
    """Upstream dpfm/utils.py::WeightedBCELoss: padded zeros count
    as negatives, weights from the positive fraction of `gt`."""

    def forward(self, prediction: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
        class_loss = F.binary_cross_entropy(prediction, gt, reduction="none")
        weights = torch.ones_like(gt)
        w_negative = gt.sum() / gt.size(0)
        w_positive = 1 - w_negative
        weights[gt >= 0.5] = w_positive
        weights[gt < 0.5] = w_negative
        return torch.mean(weights * class_loss)


class FrobeniusLoss(nn.Module):
    """utils/loss.py:8-15 (overrides the upstream import)."""

    def forward(self, a, b):
        loss = torch.sum((a - b) ** 2, axis=(1, 2))
        loss = torch.clamp(loss, min=-1, max=1000)
        return torch.mean(loss)
