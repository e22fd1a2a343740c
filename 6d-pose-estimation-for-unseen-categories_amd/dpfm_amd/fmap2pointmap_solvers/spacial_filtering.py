"""Top-5 + pairwise-rigidity point-map solver (reference
fmap2pointmap_solvers/spacial_filtering.py:5-75) on the HIP feature-distance (top-5
epilogue) and rigidity-filter kernels."""
from __future__ import annotations

import torch

from .. import ops

K = 5


def nn_query(feat_x, feat_y, dim=-2):
    """5 nearest rows of feat_x for every row of feat_y, PC-major: int64 [2, 5*V2]."""
    V1, V2 = feat_x.shape[0], feat_y.shape[0]
    dev = feat_x.device
    eye = torch.eye(30, dtype=torch.float32, device=dev)[None]
    n1 = torch.tensor([V1], dtype=torch.int32, device=dev)
    n2 = torch.tensor([V2], dtype=torch.int32, device=dev)
    idx, _ = ops.feat_dist_topk(feat_x[None].float(), eye, feat_y[None].float(), n1, n2, K)
    idx = idx[0]
    idx_p = torch.arange(V2, device=dev, dtype=torch.int64)[:, None].expand(V2, K)
    return torch.stack([idx, idx_p], 0).reshape(2, -1)


def spacial_filtering(CAD, PC, p_pred, diam_cad):
    """Three rigidity rounds (spacial_filtering.py:42-75). CAD [V1,3], PC [V2,3] f32,
    p_pred int64 [2, n]; returns the surviving columns of p_pred."""
    dev = CAD.device
    n = p_pred.shape[1]
    cand = p_pred.t().contiguous()[None]
    ncand = torch.tensor([n], dtype=torch.int32, device=dev)
    thr4 = ops.rigidity_thresholds([float(diam_cad)], dev)
    rows, cnt = ops.rigidity_filter(cand, ncand, CAD.float()[None], PC.float()[None], thr4)
    keep = rows[0, :int(cnt[0].item())]
    return p_pred[:, keep]


def spacial_filtering_fmap2pointmap(C12, evecs_x, evecs_y, CAD, PC, diam_cad):
    if C12.dim() == 3:
        C12 = C12.squeeze(0)
    V1, V2 = evecs_x.shape[0], evecs_y.shape[0]
    dev = evecs_x.device
    n1 = torch.tensor([V1], dtype=torch.int32, device=dev)
    n2 = torch.tensor([V2], dtype=torch.int32, device=dev)
    idx, _ = ops.feat_dist_topk(evecs_x[None].float(), C12[None].float(), evecs_y[None].float(), n1, n2, K)
    idx_p = torch.arange(V2, device=dev, dtype=torch.int64)[:, None].expand(V2, K)
    pp = torch.stack([idx[0], idx_p], 0).reshape(2, -1)
    return spacial_filtering(CAD, PC, pp, diam_cad)
