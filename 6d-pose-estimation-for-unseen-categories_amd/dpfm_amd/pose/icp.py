"""ICP refinement after RANSAC — the (f4) row: scripts/test_RANSAC.py:436-446 runs Open3D
0.17 `registration_icp(source = CAD, target = CAD posed by T_gt, threshold = 0.2, trans_init =
T_RANSAC, TransformationEstimationPointToPoint(), ICPConvergenceCriteria(max_iteration=2000))`.

`registration_icp` keeps that signature (numpy or tensors in, a RegistrationResult out);
`refine_to_crop` is the variant the reference does not offer: ICP of the CAD against the
OBSERVED crop (camera frame), which needs no ground truth. The reference's target (the
GT-posed CAD) makes its "after ICP" numbers an upper bound; see DESIGN.md §7.

Semantics (csrc/icp.hip, parity unpinned against Open3D): nearest target point by exact fp64
distance (ties: lowest index), pair iff d^2 < threshold^2, Umeyama without scaling, stop on
|dfitness| < 1e-6 and |drmse| < 1e-6 or after max_iteration updates."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .. import ops


@dataclass
class ICPResult:
    """The fields of open3d.pipelines.registration.RegistrationResult the reference reads,
    plus the iteration count and whether the relative criteria stopped the loop."""
    transformation: np.ndarray
    fitness: float
    inlier_rmse: float
    iterations: int
    converged: bool


def _dev(device):
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


def _f64(x, dev):
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=torch.float64).contiguous()
    return torch.as_tensor(np.asarray(x, dtype=np.float64), device=dev).contiguous()


def registration_icp(source, target, max_correspondence_distance, init=None, max_iteration: int = 30,
                     relative_fitness: float = 1e-6, relative_rmse: float = 1e-6, device=None) -> ICPResult:
    """source [Ns,3], target [Nt,3], init 4x4 (identity if None) -> ICPResult (one crop)."""
    dev = _dev(device)
    src = _f64(source, dev).reshape(-1, 3)
    tgt = _f64(target, dev).reshape(-1, 3)
    T0 = _f64(np.eye(4) if init is None else init, dev).reshape(1, 4, 4)
    so = torch.tensor([0, src.shape[0]], dtype=torch.int64, device=dev)
    to = torch.tensor([0, tgt.shape[0]], dtype=torch.int64, device=dev)
    T, st = ops.icp(src, so, tgt, to, T0, max_correspondence_distance, max_iteration, relative_fitness,
                    relative_rmse, nsrc_max=src.shape[0], ntgt_max=tgt.shape[0])
    st = st[0].cpu().numpy()
    return ICPResult(T[0].cpu().numpy(), float(st[0]), float(st[1]), int(st[2]), bool(st[3]))


def icp_batched(src, src_off, tgt, tgt_off, T_init, max_dist: float = 0.2, max_iter: int = 2000,
                rel_fitness: float = 1e-6, rel_rmse: float = 1e-6, nsrc_max=None, ntgt_max=None, poll: int = 8):
    """All crops at once (device tensors, packed layout): (T f64 [B,4,4], stats f64 [B,4])."""
    return ops.icp(src, src_off, tgt, tgt_off, T_init, max_dist, max_iter, rel_fitness, rel_rmse,
                   nsrc_max=nsrc_max, ntgt_max=ntgt_max, poll=poll)


def gt_posed_target(cad, off, T_gt):
    """The reference's ICP target (test_RANSAC.py:426-427, 436): every crop's CAD under T_gt,
    packed like `cad` (f64 [T,3]); `transform` of test_RANSAC.py:154-160 (pcd @ R^T + t)."""
    B = off.numel() - 1
    counts = (off[1:] - off[:-1])
    crop = torch.repeat_interleave(torch.arange(B, device=cad.device), counts)
    R = T_gt[:, :3, :3].to(torch.float64)[crop]
    t = T_gt[:, :3, 3].to(torch.float64)[crop]
    return (torch.einsum("nc,nrc->nr", cad.to(torch.float64), R) + t).contiguous()


def refine_to_crop(cad, cad_off, crop, crop_off, T_ransac, max_dist: float = 0.2, max_iter: int = 2000, **kw):
    """ICP of each crop's CAD (object frame) against its observed crop points (camera frame),
    starting from the RANSAC pose: (T f64 [B,4,4], stats f64 [B,4])."""
    return ops.icp(cad, cad_off, crop, crop_off, T_ransac, max_dist, max_iter, **kw)
