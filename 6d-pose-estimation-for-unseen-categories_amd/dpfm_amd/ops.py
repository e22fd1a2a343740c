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
