"""Torch-tensor front-ends of the libposekern C-ABI (device tensors only, stream-ordered
on torch's current stream, no host synchronisation unless a function says so).

Ragged batches use the packed layout of include/posekern.h: per-crop rows are
concatenated and `offsets[b] .. offsets[b+1]` delimits crop b (int64, on device).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr

_I = lambda v: int(v)  # noqa: E731


def _dev(t: torch.Tensor) -> torch.device:
    return t.device


# ------------------------------------------------------------------------------ H3 FPS


def fps_packed(xyz: torch.Tensor, offsets: torch.Tensor, nmax: int, start: torch.Tensor,
               npoint: torch.Tensor, out_stride: int) -> torch.Tensor:
    """Farthest point sampling of B packed crops (pk_fps).

    xyz f32 [T,3]; offsets int64 [B+1]; start/npoint int32 [B]; returns int64
    [B, out_stride] (row b valid for its first npoint[b] entries).
    """
    assert xyz.dtype == torch.float32 and xyz.dim() == 2 and xyz.shape[1] == 3
    B = offsets.numel() - 1
    out = torch.zeros((B, out_stride), dtype=torch.int64, device=xyz.device)
    call("pk_fps", ptr(xyz), ptr(offsets), B, int(nmax), ptr(start.to(torch.int32).contiguous()),
         ptr(npoint.to(torch.int32).contiguous()), ptr(out), int(out_stride), _lib.stream(xyz.device))
    return out


# ------------------------------------------------------------------------------ H5 ball query


def ball_threshold(r: float) -> float:
    """Largest double s with sqrt_rn(s) <= r, so that `s <= T(r)` == `sqrt(s) <= r`
    exactly (np.linalg.norm(...) <= r at dataset/object.py:283-286)."""
    r = float(r)
    if not (r >= 0.0) or math.isinf(r):
        return r * r if r >= 0 else -1.0
    s = r * r
    while s > 0 and math.sqrt(s) > r:
        s = math.nextafter(s, -math.inf)
    while math.sqrt(math.nextafter(s, math.inf)) <= r:
        s = math.nextafter(s, math.inf)
    return s


def ball_query(cad: torch.Tensor, cad_off: torch.Tensor, pc: torch.Tensor, pc_off: torch.Tensor,
               radius: Sequence[float] | torch.Tensor, n1max: int, n2max: int, cap: int,
               with_mask: bool = True, thr2: Optional[torch.Tensor] = None) -> dict:
    """find_positives for B packed crop pairs (pk_ball_query_mask + pk_ball_query_pairs).

    Returns dict(mask uint8 [B,n1max,ld] or None, rowcount int32 [B,n1max], pairs int64
    [B,cap,2], count int64 [B], overlap_12 int8 [B,n1max], overlap_21 int8 [B,n2max]).
    count[b] > cap means the pair list of crop b was truncated (check_capacity raises).
    """
    assert cad.dtype == torch.float64 and pc.dtype == torch.float64
    dev = cad.device
    B = cad_off.numel() - 1
    if thr2 is None:
        r = radius.tolist() if isinstance(radius, torch.Tensor) else list(radius)
        thr2 = torch.tensor([ball_threshold(x) for x in r], dtype=torch.float64, device=dev)
    ld = ((n2max + 15) // 16) * 16
    mask = torch.empty((B, n1max, ld), dtype=torch.uint8, device=dev) if with_mask else None
    rowcount = torch.empty((B, n1max), dtype=torch.int32, device=dev)
    s = _lib.stream(dev)
    call("pk_ball_query_mask", ptr(cad), ptr(cad_off), ptr(pc), ptr(pc_off), ptr(thr2), B, int(n1max),
         int(n2max), ptr(mask), int(ld), ptr(rowcount), s)
    rowoff = torch.empty((B, n1max), dtype=torch.int64, device=dev)
    pairs = torch.empty((B, cap, 2), dtype=torch.int64, device=dev)
    count = torch.empty((B,), dtype=torch.int64, device=dev)
    ov12 = torch.empty((B, n1max), dtype=torch.int8, device=dev)
    ov21 = torch.empty((B, n2max), dtype=torch.int8, device=dev)
    call("pk_ball_query_pairs", ptr(cad), ptr(cad_off), ptr(pc), ptr(pc_off), ptr(thr2), B, int(n1max),
         int(n2max), ptr(mask), int(ld), ptr(rowcount), ptr(rowoff), ptr(pairs), int(cap), ptr(count),
         ptr(ov12), ptr(ov21), s)
    return dict(mask=mask, rowcount=rowcount, pairs=pairs, count=count, overlap_12=ov12, overlap_21=ov21,
                thr2=thr2)


def check_capacity(count: torch.Tensor, cap: int, what: str = "pairs") -> None:
    """Host-synchronising overflow check for capacity/count outputs."""
    m = int(count.max().item()) if count.numel() else 0
    if m > cap:
        raise _lib.PoseKernError(f"{what}: {m} entries exceed capacity {cap}; re-run with cap >= {m}")


def packed_offsets(sizes: Sequence[int], device) -> torch.Tensor:
    off = np.zeros(len(sizes) + 1, dtype=np.int64)
    off[1:] = np.cumsum(np.asarray(sizes, dtype=np.int64))
    return torch.from_numpy(off).to(device)


# ------------------------------------------------------------------------------ H1 / H2 / H4 crops


def backproject(depth: torch.Tensor, mask: torch.Tensor, K: torch.Tensor, cam_scale: torch.Tensor,
                cap: int) -> dict:
    """dpt_2_pcld for F frames (pk_backproject). depth uint16 [F,H,W] (int16 storage),
    mask uint8 [F,H,W], K f64 [F,9], cam_scale f32 [F]. Returns packed xyz f64 [cap,3],
    count int64 [F], off int64 [F+1] (count > cap overflows; see check_capacity)."""
    F, H, W = depth.shape
    dev = depth.device
    rowcnt = torch.empty((F, H), dtype=torch.int32, device=dev)
    rowoff = torch.empty((F, H), dtype=torch.int64, device=dev)
    count = torch.empty((F,), dtype=torch.int64, device=dev)
    off = torch.empty((F + 1,), dtype=torch.int64, device=dev)
    xyz = torch.empty((cap, 3), dtype=torch.float64, device=dev)
    call("pk_backproject", ptr(depth), ptr(mask), F, H, W, ptr(K), ptr(cam_scale), ptr(rowcnt), ptr(rowoff),
         ptr(count), ptr(off), ptr(xyz), int(cap), _lib.stream(dev))
    return dict(xyz=xyz, count=count, off=off)


def sor(xyz: torch.Tensor, off: torch.Tensor, nmax: int, knn: int = 20, std_ratio: float = 0.3,
        want64: bool = True, want32: bool = True, want_idx: bool = False) -> dict:
    """remove_outliers for B packed crops (pk_sor). Survivors are packed by out_off."""
    B = off.numel() - 1
    dev = xyz.device
    T = xyz.shape[0]
    nchunk = max(1, (nmax + 1023) // 1024)
    avg = torch.empty((T,), dtype=torch.float64, device=dev)
    thr = torch.empty((B,), dtype=torch.float64, device=dev)
    ccount = torch.empty((B, nchunk), dtype=torch.int32, device=dev)
    coff = torch.empty((B, nchunk), dtype=torch.int64, device=dev)
    kept = torch.empty((B,), dtype=torch.int64, device=dev)
    out_off = torch.empty((B + 1,), dtype=torch.int64, device=dev)
    out64 = torch.empty((T, 3), dtype=torch.float64, device=dev) if want64 else None
    out32 = torch.empty((T, 3), dtype=torch.float32, device=dev) if want32 else None
    kidx = torch.empty((T,), dtype=torch.int64, device=dev) if want_idx else None
    call("pk_sor", ptr(xyz), ptr(off), B, int(nmax), int(knn), float(std_ratio), ptr(avg), ptr(thr), ptr(ccount),
         ptr(coff), ptr(kept), ptr(out_off), ptr(out64), ptr(out32), ptr(kidx), _lib.stream(dev))
    return dict(avg=avg, thr=thr, kept=kept, off=out_off, xyz64=out64, xyz32=out32, kept_idx=kidx)


def fps_npoint(off: torch.Tensor, fixed: int = 0, limit: int = 2000, seed: int = 0) -> dict:
    B = off.numel() - 1
    dev = off.device
    npoint = torch.empty((B,), dtype=torch.int32, device=dev)
    start = torch.empty((B,), dtype=torch.int32, device=dev)
    out_off = torch.empty((B + 1,), dtype=torch.int64, device=dev)
    call("pk_fps_npoint", ptr(off), B, int(fixed), int(limit), ctypes_u64(seed), ptr(npoint), ptr(start),
         ptr(out_off), _lib.stream(dev))
    return dict(npoint=npoint, start=start, off=out_off)


def ctypes_u64(v: int):
    import ctypes
    return ctypes.c_uint64(int(v) & 0xFFFFFFFFFFFFFFFF)


def gather_transform(pcd: torch.Tensor, off: torch.Tensor, idx: Optional[torch.Tensor], npoint: torch.Tensor,
                     npmax: int, out_off: torch.Tensor, R: torch.Tensor, t: torch.Tensor, total_cap: int,
                     want_sel64: bool = True, want_align: bool = True, want_sel32: bool = True) -> dict:
    B = off.numel() - 1
    dev = pcd.device
    sel64 = torch.empty((total_cap, 3), dtype=torch.float64, device=dev) if want_sel64 else None
    align = torch.empty((total_cap, 3), dtype=torch.float64, device=dev) if want_align else None
    sel32 = torch.empty((total_cap, 3), dtype=torch.float32, device=dev) if want_sel32 else None
    idx_stride = idx.shape[1] if idx is not None else 0
    call("pk_gather_transform", ptr(pcd), ptr(off), B, ptr(idx), int(idx_stride), ptr(npoint), int(npmax),
         ptr(out_off), ptr(R), ptr(t), ptr(sel64), ptr(align), ptr(sel32), _lib.stream(dev))
    return dict(sel64=sel64, align=align, sel32=sel32)
