"""Crop formation with the reference's dataset API (dataset/object.py), on the device.

The reference runs these steps per crop inside DataLoader worker processes on the
CPU (numpy + OpenCV + Open3D + a torch FPS loop) and caches the results in .npz files.
Here each function keeps its reference name, arguments and return meaning, but the
work runs in libposekern (`ops`), and `CropFormation` runs the whole chain for a batch
of frames in one stream-ordered sequence with no host synchronisation:

  dpt_2_pcld (+erode_seg_mask)  :73-88, :52-71   -> pk_backproject / pk_erode_mask
  remove_outliers               :33-50           -> pk_sor
  farthest_point_sample policy  :145-148         -> pk_fps_npoint + pk_fps
  pcd[idx0], transform(inv)     :148, :174, :304 -> pk_gather_transform
  find_positives, get_overlap   :177-180, :281-317 -> pk_ball_query_mask/_pairs
  (RGB at the crop points: H16) -> pk_sample_rgb
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .. import ops


def _dev(device):
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


def _to_np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()


# ----------------------------------------------------------------------------- per-crop API


def erode_seg_mask(mask, kernel_size=3, device=None):
    """Plus-shaped 3x3 erosion of a boolean mask (object.py:52-71). numpy in -> numpy out."""
    if kernel_size != 3:
        raise ValueError("the reference erodes with a 3x3 plus kernel (object.py:80)")
    dev = _dev(device)
    m = torch.as_tensor(np.where(np.asarray(mask, dtype=bool), 255, 0).astype(np.uint8), device=dev)[None]
    return _to_np(ops.erode_mask(m)[0]).astype(bool)


def dpt_2_pcld(dpt, cam_scale, K, mask, device=None):
    """Back-project the eroded mask of a depth image to points in cm (object.py:73-88).
    dpt uint16 [H, W] (or [H, W, C]: channel 0), cam_scale = 1000 / depth_scale, K 3x3,
    mask bool [H, W]. Returns f64 [P, 3] in row-major pixel order."""
    dev = _dev(device)
    dpt = np.asarray(dpt)
    if dpt.ndim > 2:
        dpt = dpt[:, :, 0]
    H, W = dpt.shape
    depth = torch.as_tensor(dpt.astype(np.uint16).view(np.int16), device=dev)[None]
    m = torch.as_tensor(np.where(np.asarray(mask, dtype=bool), 255, 0).astype(np.uint8), device=dev)[None]
    Kt = torch.as_tensor(np.asarray(K, dtype=np.float64).reshape(1, 9), device=dev)
    cs = torch.tensor([np.float32(cam_scale)], dtype=torch.float32, device=dev)
    out = ops.backproject(depth, m, Kt, cs, cap=H * W)
    n = int(out["count"][0].item())
    return _to_np(out["xyz"][:n])


def remove_outliers(pcd, device=None):
    """Statistical outlier removal, nb_neighbors = 20, std_ratio = 0.3 (object.py:33-50)."""
    dev = _dev(device)
    x = torch.as_tensor(np.asarray(pcd, dtype=np.float64), device=dev).contiguous()
    off = torch.tensor([0, x.shape[0]], dtype=torch.int64, device=dev)
    res = ops.sor(x, off, x.shape[0], 20, 0.3, want64=True, want32=False)
    n = int(res["kept"][0].item())
    return _to_np(res["xyz64"][:n])


def transform(pc, R, t, inv=False, device=None):
    """object.py:304-309: pc @ R + (-t @ R) if inv (object frame), else pc @ R.T + t."""
    pc = np.asarray(pc, dtype=np.float64)
    R = np.asarray(R, dtype=np.float64).reshape(3, 3)
    t = np.asarray(t, dtype=np.float64).reshape(3)
    if not inv:  # pc @ R.T + t is the inverse form with R' = R^T, t' = -t @ R
        R, t = R.T.copy(), -(t @ R)
    dev = _dev(device)
    x = torch.as_tensor(pc, device=dev).contiguous()
    n = x.shape[0]
    off = torch.tensor([0, n], dtype=torch.int64, device=dev)
    npoint = torch.tensor([-n], dtype=torch.int32, device=dev)
    g = ops.gather_transform(x, off, None, npoint, n, off, torch.as_tensor(R.reshape(1, 9), device=dev),
                             torch.as_tensor(t.reshape(1, 3), device=dev), n, want_sel64=False, want_sel32=False)
    return _to_np(g["align"])


def find_positives(pc1, pc2, r=0.2, device=None, cap: Optional[int] = None):
    """All (i, j) with ||pc1[i] - pc2[j]|| <= r, row-major (object.py:281-288), bit-exact."""
    dev = _dev(device)
    a = torch.as_tensor(np.asarray(pc1, dtype=np.float64), device=dev).contiguous()
    b = torch.as_tensor(np.asarray(pc2, dtype=np.float64), device=dev).contiguous()
    n1, n2 = a.shape[0], b.shape[0]
    cap = cap or max(1, n1 * min(n2, 256))
    while True:
        res = ops.ball_query(a, torch.tensor([0, n1], device=dev), b, torch.tensor([0, n2], device=dev), [r], n1, n2,
                             cap, with_mask=False)
        c = int(res["count"][0].item())
        if c <= cap:
            return _to_np(res["pairs"][0, :c])
        cap = c


def get_overlap(l_1, l_2, p):
    """object.py:311-317: int8 "has a partner" masks from a pair list."""
    p = np.asarray(p)
    o12 = np.zeros((l_1,), dtype=np.byte)
    o21 = np.zeros((l_2,), dtype=np.byte)
    if p.size:
        o12[p[:, 0]] = 1
        o21[p[:, 1]] = 1
    return o12, o21


# ----------------------------------------------------------------------------- batched chain


@dataclass
class FrameBatch:
    """RGB-D frames + per-object data resident in device memory (one crop per frame)."""
    depth: torch.Tensor      # int16 [F, H, W] (uint16 bits)
    mask: torch.Tensor       # uint8 [F, H, W] mask_visib values (255 = object)
    rgb: torch.Tensor        # uint8 [F, H, W, 3]
    K: torch.Tensor          # f64 [F, 9]
    cam_scale: torch.Tensor  # f32 [F] = 1000 / depth_scale
    R: torch.Tensor          # f64 [F, 9] R_m2c row-major
    t: torch.Tensor          # f64 [F, 3] t_m2c (cm)
    cad64: torch.Tensor      # f64 [sum N1_f, 3] CAD vertices (cm), packed
    cad_off: torch.Tensor    # int64 [F + 1]
    diam: list               # host floats (cm), models_info diameter * 0.1
    max_pixels: int          # host bound on mask pixels per frame (kernel grid sizing)
    thr2: torch.Tensor       # f64 [F] ball-query threshold T(0.05 * diam) (ops.ball_threshold)
    n1max: int = 0           # largest CAD (collate's padded CAD length)


@dataclass
class Crops:
    """One batch of formed crops. Packed fields hold crop b in rows off[b]..off[b+1]; the
    model-facing fields are collate's zero-padded [F, ld, .] layout (dataset/helpers.py:22-50)."""
    pc64: torch.Tensor       # f64 packed [*, 3] crop points, camera frame (pcd_depth)
    pc32: torch.Tensor       # f32 [F, ld, 3] PC xyz fed to the model (object.py:263), zero-padded
    align64: torch.Tensor    # f64 packed [*, 3] crop in the object frame (align_pc)
    align32: torch.Tensor    # f32 [F, ld, 3] Obj["align_pc"] after collate
    off: torch.Tensor        # int64 [F + 1] packed offsets of the crops
    n2: torch.Tensor         # int32 [F] points per crop (the rows of pc32 that are not padding)
    ld: int                  # padded crop length (the batch maximum when pad="batch")
    npoint: torch.Tensor     # int32 [F] FPS policy (negative: every point kept, no FPS)
    pairs: torch.Tensor      # int64 [F, cap, 2] P (CAD idx, PC idx), row-major
    npairs: torch.Tensor     # int64 [F] true pair counts (> pair_cap: truncated, see overflow)
    overlap_12: torch.Tensor  # int8 [F, N1max]
    overlap_21: torch.Tensor  # int8 [F, ld]
    rgb: Optional[torch.Tensor]  # f32 [*, C] colour at each packed crop point (H16) or None
    kept: torch.Tensor       # int64 [F] points after outlier removal
    pair_cap: int = 0
    overflow_flag: Optional[torch.Tensor] = None  # 0-d int32 formed with the crops (see overflow)
    # f32 [F, k, k] ground-truth functional map (utils/utils.py:67-79) when the producer formed it
    # beside the crops (PipelinedTrainer: on the crop-formation stream); None: the step solves it
    C_gt: Optional[torch.Tensor] = None
    # int32 [F] per crop 1 when an FPS index fell outside its crop (pk_gather_transform's check;
    # those points are NaN): checked by check(), never read on the step's path
    index_status: Optional[torch.Tensor] = None
    # int32 [F, ld] pairs per crop point among the kept P (pk_ball_query_pairs' colcount): C_gt's
    # row weights, formed with the crops so the step's C_gt needs no count launches
    pair_cols: Optional[torch.Tensor] = None

    def overflow(self) -> torch.Tensor:
        """0-d flag on the device (nonzero: some crop had more ball-query pairs than pair_cap, its
        P was truncated; pk_ball_query_pairs forms it). No host sync; `check()` raises on it. CropFormation forms it on its
        own stream, so the training step only reads it."""
        if self.overflow_flag is not None:
            return self.overflow_flag
        return (self.npairs > self.pair_cap).any()

    def check(self) -> None:
        """Host-synchronising: raise if a pair list overflowed its capacity or an FPS index was
        out of range."""
        ops.check_capacity(self.npairs, self.pair_cap, "ball-query pairs (CropFormation pair_cap)")
        ops.check_index_status(self.index_status, "CropFormation (FPS indices)")


class CropFormation:
    """Frames -> model-ready crops for a whole batch, with the reference's sample policy
    (dataset/object.py:145-148) and collate's padding (dataset/helpers.py:22-50).

    npoint = 0: the reference policy — FPS to int(2000/n*n) points (1999 or 2000) when the
    crop has more than `limit` = 2000 points, every point otherwise (ragged crops).
    npoint > 0: a fixed target — FPS to exactly `npoint` when the crop is larger, every
    point otherwise (the benchmark configs' 1024 / 2048 / 4096-point crops).

    pad = "batch": pad to the largest crop of the batch, exactly collate's pad_sequence
    (one host read of the per-crop counts; eager use). pad = "fixed": pad to the policy's
    maximum (npoint, or `limit`), no host synchronisation (HIP-graph capture); identical to
    collate whenever some crop reaches that maximum, otherwise the model sees more zero
    padding than the reference would. Default: "fixed" for npoint > 0, "batch" for 0."""

    def __init__(self, n1: int = 0, npoint: int = 1024, pair_cap: Optional[int] = None, seed: int = 0,
                 with_mask: bool = True, pad: Optional[str] = None, limit: int = 2000, with_rgb: bool = False,
                 base: int = 0):
        self.n1, self.npoint, self.limit = n1, npoint, limit
        self.base = base  # global index of this batch's first crop (FPS start draws of a rank's shard)
        self.npmax = npoint if npoint > 0 else limit
        self.pair_cap = pair_cap or 64 * self.npmax
        self.seed = seed
        self.with_mask = with_mask
        self.pad = pad or ("fixed" if npoint > 0 else "batch")
        if self.pad not in ("batch", "fixed"):
            raise ValueError("pad must be 'batch' or 'fixed'")
        self.with_rgb = with_rgb

    def __call__(self, fb: FrameBatch) -> Crops:
        F_, H, W = fb.depth.shape
        bp = ops.backproject(fb.depth, fb.mask, fb.K, fb.cam_scale, cap=F_ * fb.max_pixels)
        so = ops.sor(bp["xyz"], bp["off"], fb.max_pixels, 20, 0.3, pix=bp["pix"], idxmap=bp["idxmap"], K=fb.K,
                     want64=True, want32=True)
        pol = ops.fps_npoint(so["off"], fixed=self.npoint, limit=self.limit, seed=self.seed, base=self.base)
        npmax = self.npmax
        if self.pad == "batch":  # collate pads to the batch maximum: read it (host sync)
            ld = int((pol["off"][1:] - pol["off"][:-1]).max().item()) if F_ > 0 else 0
        else:
            ld = npmax
        idx = ops.fps_packed(so["xyz32"], so["off"], fb.max_pixels, pol["start"], pol["npoint"], npmax)
        st = torch.empty((F_,), dtype=torch.int32, device=fb.depth.device)
        # PC["xyz"] = f32(pcd) and Obj["align_pc"], padded as collate does, in the gather's launch
        g = ops.gather_transform(so["xyz64"], so["off"], idx, pol["npoint"], npmax, pol["off"], fb.R, fb.t,
                                 F_ * npmax, want_sel32=False, status=st, pad_ld=ld)
        pc32, n2, align32 = g["pc32"], g["n2"], g["align32"]
        n1max = fb.n1max or self.n1
        bq = ops.ball_query(fb.cad64, fb.cad_off, g["align"], pol["off"], None, n1max, ld, self.pair_cap,
                            with_mask=self.with_mask, thr2=fb.thr2)
        rgb = ops.sample_rgb(fb.rgb, fb.K, g["sel64"], pol["off"], npmax) if self.with_rgb else None
        return Crops(pc64=g["sel64"], pc32=pc32, align64=g["align"], align32=align32, off=pol["off"], n2=n2, ld=ld,
                     npoint=pol["npoint"], pairs=bq["pairs"], npairs=bq["count"], overlap_12=bq["overlap_12"],
                     overlap_21=bq["overlap_21"], rgb=rgb, kept=so["kept"], pair_cap=self.pair_cap,
                     overflow_flag=bq["overflow"], index_status=st, pair_cols=bq["colcount"])
