"""Torch-tensor front-ends of the libposekern C-ABI (device tensors only, stream-ordered
on torch's current stream, no host synchronisation unless a function says so).

Ragged batches use the packed layout of include/posekern.h: per-crop rows are
concatenated and `offsets[b] .. offsets[b+1]` delimits crop b (int64, on device).
"""
from __future__ import annotations

import ctypes
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
    out = torch.empty((B, out_stride), dtype=torch.int64, device=xyz.device)  # the kernel zero-fills the tails
    call("pk_fps", ptr(xyz), ptr(offsets), B, int(nmax), ptr(start.to(torch.int32).contiguous()),
         ptr(npoint.to(torch.int32).contiguous()), ptr(out), int(out_stride), _lib.stream(xyz.device),
         work=("hbm", 12 * xyz.shape[0] + 8 * B * int(out_stride)))
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
               with_mask: bool = True, thr2: Optional[torch.Tensor] = None, colcount: bool = True) -> dict:
    """find_positives for B packed crop pairs (pk_ball_query_mask + pk_ball_query_pairs).

    Returns dict(mask uint8 [B,n1max,ld] or None, rowcount int32 [B,n1max], pairs int64
    [B,cap,2], count int64 [B], overlap_12 int8 [B,n1max], overlap_21 int8 [B,n2max],
    colcount int32 [B,n2max] or None: pairs per crop point among the kept list, C_gt's row weights).
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
         int(n2max), ptr(mask), int(ld), ptr(rowcount), s,
         work=("hbm", 24 * (cad.shape[0] + pc.shape[0]) + B * int(n1max) * int(n2max) + 4 * B * int(n1max)))
    rowoff = torch.empty((B, n1max), dtype=torch.int64, device=dev)
    pairs = torch.empty((B, cap, 2), dtype=torch.int64, device=dev)
    count = torch.empty((B,), dtype=torch.int64, device=dev)
    ov12 = torch.empty((B, n1max), dtype=torch.int8, device=dev)
    ov21 = torch.empty((B, n2max), dtype=torch.int8, device=dev)
    over = torch.empty((1,), dtype=torch.int32, device=dev)
    cc = torch.empty((B, n2max), dtype=torch.int32, device=dev) if colcount else None
    call("pk_ball_query_pairs", ptr(cad), ptr(cad_off), ptr(pc), ptr(pc_off), ptr(thr2), B, int(n1max),
         int(n2max), ptr(mask), int(ld), ptr(rowcount), ptr(rowoff), ptr(pairs), int(cap), ptr(count),
         ptr(ov12), ptr(ov21), ptr(over), ptr(cc), s)
    return dict(mask=mask, rowcount=rowcount, pairs=pairs, count=count, overlap_12=ov12, overlap_21=ov21,
                thr2=thr2, overflow=over[0], colcount=cc)


def check_index_status(status: Optional[torch.Tensor], what: str) -> None:
    """Host-synchronising check of an index consumer's per-crop status (pk_inlier_ratio,
    pk_gather_transform, pk_ransac: 1 = an index outside its array was met; the kernel did not
    read through it). Raises PoseKernError naming the crops."""
    if status is None or status.numel() == 0:
        return
    bad = torch.nonzero(status).flatten()
    if bad.numel():
        raise _lib.PoseKernError(f"{what}: out-of-range index in crop(s) {bad[:8].tolist()}"
                                 f"{' ...' if bad.numel() > 8 else ''}")


def _index_status(B: int, dev, status: Optional[torch.Tensor], check: Optional[bool]):
    """(status buffer to pass, whether to check it after the call): a caller-given buffer is
    written and left to the caller; otherwise a temporary one is checked right after the call
    (host sync) unless a HIP graph is being captured (no check, nothing to hold it)."""
    if status is not None:
        return status, bool(check)
    if torch.cuda.is_current_stream_capturing():
        return None, False
    return torch.empty((B,), dtype=torch.int32, device=dev), check is None or bool(check)


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
    pix = torch.empty((cap,), dtype=torch.int32, device=dev)
    idxmap = torch.empty((F, H, W), dtype=torch.int32, device=dev)
    call("pk_backproject", ptr(depth), ptr(mask), F, H, W, ptr(K), ptr(cam_scale), ptr(rowcnt), ptr(rowoff),
         ptr(count), ptr(off), ptr(xyz), int(cap), ptr(pix), ptr(idxmap), _lib.stream(dev),
         work=("hbm", 7 * F * H * W))
    return dict(xyz=xyz, count=count, off=off, pix=pix, idxmap=idxmap)


def sor(xyz: torch.Tensor, off: torch.Tensor, nmax: int, knn: int = 20, std_ratio: float = 0.3,
        want64: bool = True, want32: bool = True, want_idx: bool = False, pix: Optional[torch.Tensor] = None,
        idxmap: Optional[torch.Tensor] = None, K: Optional[torch.Tensor] = None) -> dict:
    """remove_outliers for B packed crops (pk_sor). Survivors are packed by out_off.
    pix/idxmap (from backproject) enable the exact pixel-window kNN bound; with the frames'
    intrinsics K (f64 [B, 9]) only the pixel box that can hold a neighbour is scanned."""
    if K is not None:
        K = K.to(dtype=torch.float64).reshape(-1, 9).contiguous()
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
    H = idxmap.shape[1] if idxmap is not None else 0
    W = idxmap.shape[2] if idxmap is not None else 0
    call("pk_sor", ptr(xyz), ptr(off), B, int(nmax), int(knn), float(std_ratio), ptr(pix), ptr(idxmap), H, W,
         ptr(K), ptr(avg), ptr(thr), ptr(ccount),
         ptr(coff), ptr(kept), ptr(out_off), ptr(out64), ptr(out32), ptr(kidx), _lib.stream(dev),
         work=("hbm", 68 * xyz.shape[0]))
    return dict(avg=avg, thr=thr, kept=kept, off=out_off, xyz64=out64, xyz32=out32, kept_idx=kidx)


def fps_npoint(off: torch.Tensor, fixed: int = 0, limit: int = 2000, seed: int = 0, base: int = 0) -> dict:
    B = off.numel() - 1
    dev = off.device
    npoint = torch.empty((B,), dtype=torch.int32, device=dev)
    start = torch.empty((B,), dtype=torch.int32, device=dev)
    out_off = torch.empty((B + 1,), dtype=torch.int64, device=dev)
    call("pk_fps_npoint", ptr(off), B, int(fixed), int(limit), ctypes_u64(seed), int(base), ptr(npoint), ptr(start),
         ptr(out_off), _lib.stream(dev))
    return dict(npoint=npoint, start=start, off=out_off)


def ctypes_u64(v: int):
    import ctypes
    return ctypes.c_uint64(int(v) & 0xFFFFFFFFFFFFFFFF)


def collate_pad(src: torch.Tensor, off: torch.Tensor, ld: int) -> tuple[torch.Tensor, torch.Tensor]:
    """collate (dataset/helpers.py:22-50) of one packed field on the device (pk_collate_pad):
    src f64 / f32 [T, C] packed by off [B+1] -> (f32 [B, ld, C] zero-padded, counts int32 [B]).
    ld = the batch maximum count reproduces collate's pad_sequence exactly."""
    if src.dtype not in (torch.float32, torch.float64):
        raise _lib.PoseKernError("collate_pad: f32 / f64 sources only")
    src2 = src.reshape(src.shape[0], -1) if src.dim() != 1 else src[:, None]
    C = int(src2.shape[1]) if src2.dim() == 2 and src2.shape[1] > 0 else 1
    B = off.numel() - 1
    dev = off.device
    dst = torch.empty((B, int(ld), C), dtype=torch.float32, device=dev)
    counts = torch.empty((B,), dtype=torch.int32, device=dev)
    if src2.numel() == 0:  # every crop empty: keep a valid pointer (no row is read)
        src2 = torch.zeros((1, C), dtype=src.dtype, device=dev)
    call("pk_collate_pad", ptr(src2.contiguous()), int(src.dtype == torch.float64), C,
         ptr(off), B, int(ld), ptr(dst) if dst.numel() else None, ptr(counts), _lib.stream(dev),
         work=("hbm", (src.element_size() + 4) * B * int(ld) * C))
    return dst, counts


def gather_transform(pcd: torch.Tensor, off: torch.Tensor, idx: Optional[torch.Tensor], npoint: torch.Tensor,
                     npmax: int, out_off: torch.Tensor, R: torch.Tensor, t: torch.Tensor, total_cap: int,
                     want_sel64: bool = True, want_align: bool = True, want_sel32: bool = True,
                     status: Optional[torch.Tensor] = None, check: Optional[bool] = None,
                     pad_ld: Optional[int] = None) -> dict:
    """pcd[idx] + transform (pk_gather_transform). status int32 [B] (optional): per crop 1 when
    an FPS index lies outside its crop (that point's outputs are NaN); without it the call checks
    a temporary one (host sync) unless capturing. Returns dict(sel64, align, sel32, status); with
    pad_ld also collate_pad's outputs of sel64 and align at ld = pad_ld in the same launch:
    pc32 / align32 f32 [B, ld, 3] and n2 int32 [B] (pk_gather_transform_pad)."""
    B = off.numel() - 1
    dev = pcd.device
    st, chk = _index_status(B, dev, status, check)
    sel64 = torch.empty((total_cap, 3), dtype=torch.float64, device=dev) if want_sel64 else None
    align = torch.empty((total_cap, 3), dtype=torch.float64, device=dev) if want_align else None
    sel32 = torch.empty((total_cap, 3), dtype=torch.float32, device=dev) if want_sel32 else None
    idx_stride = idx.shape[1] if idx is not None else 0
    if pad_ld is None:
        call("pk_gather_transform", ptr(pcd), ptr(off), B, ptr(idx), int(idx_stride), ptr(npoint), int(npmax),
             ptr(out_off), ptr(R), ptr(t), ptr(sel64), ptr(align), ptr(sel32), ptr(st), _lib.stream(dev))
        pads = {}
    else:  # collate of both fields in the same launch (pk_gather_transform_pad)
        ld = int(pad_ld)
        pc32 = torch.empty((B, ld, 3), dtype=torch.float32, device=dev)
        al32 = torch.empty((B, ld, 3), dtype=torch.float32, device=dev)
        n2 = torch.empty((B,), dtype=torch.int32, device=dev)
        call("pk_gather_transform_pad", ptr(pcd), ptr(off), B, ptr(idx), int(idx_stride), ptr(npoint), int(npmax),
             ptr(out_off), ptr(R), ptr(t), ptr(sel64), ptr(align), ptr(sel32), ptr(st), ld, ptr(pc32), ptr(al32),
             ptr(n2), _lib.stream(dev))
        pads = dict(pc32=pc32, align32=al32, n2=n2)
    if chk:
        check_index_status(st, "gather_transform (FPS indices)")
    return dict(sel64=sel64, align=align, sel32=sel32, status=st, **pads)


# ------------------------------------------------------------------------------ H7 spectral diffusion


class _SpectralDiffusion(torch.autograd.Function):
    """x_diffuse = Phi (exp(-lambda t) ⊙ (Phi^T (mass ⊙ x))) — pk_spectral_diffusion fwd/bwd.
    Gradients flow to x and t (the operators are data, as in the reference). clamp_t applies
    LearnedTimeDiffusion's in-place clamp_(min=1e-8) of t inside the kernel."""

    @staticmethod
    def forward(ctx, x, mass, evals, evecs, t, clamp_t):
        B, N, C = x.shape
        K = evecs.shape[-1]
        dev = x.device
        if x.stride(-1) != 1 or x.stride(0) != N * x.stride(1) or x.stride(1) % 4:
            x = x.contiguous()
        S = (N + 63) // 64
        work = torch.empty((B, S, K, C), dtype=torch.float32, device=dev)
        spec = torch.empty((B, K, C), dtype=torch.float32, device=dev)
        scaled = torch.empty_like(spec)
        out = torch.empty((B, N, C), dtype=torch.float32, device=dev)
        call("pk_spectral_diffusion", ptr(x), int(x.stride(1)), ptr(mass), ptr(evecs), ptr(evals), ptr(t),
             int(clamp_t), B, N, K, C, 0, ptr(work), ptr(spec), ptr(scaled), None, None, ptr(out), C, 0,
             _lib.stream(dev), work=("hbm", 16 * B * N * 64))  # Phi read twice + x in + y out, f32
        ctx.save_for_backward(mass, evals, evecs, t, spec)
        ctx.clamp_t = clamp_t
        return out

    @staticmethod
    def backward(ctx, g):
        mass, evals, evecs, t, spec = ctx.saved_tensors
        g = g.contiguous()
        B, N, C = g.shape
        K = evecs.shape[-1]
        dev = g.device
        S = (N + 63) // 64
        work = torch.empty((B, S, K, C), dtype=torch.float32, device=dev)
        scaled = torch.empty((B, K, C), dtype=torch.float32, device=dev)
        gt = torch.empty((C,), dtype=torch.float32, device=dev)
        gx = torch.empty_like(g)
        call("pk_spectral_diffusion", ptr(g), C, ptr(mass), ptr(evecs), ptr(evals), ptr(t), int(ctx.clamp_t), B, N,
             K, C, 1, ptr(work), None, ptr(scaled), ptr(spec), ptr(gt), ptr(gx), C, 0, _lib.stream(dev),
             work=("hbm", 16 * B * N * 64))
        return gx, None, None, None, gt, None


def spectral_diffusion(x, mass, evals, evecs, t, clamp_t: bool = False):
    """x [B,N,64] f32, mass [B,N], evals [B,64], evecs [B,N,64], t [64] -> [B,N,64].
    clamp_t: first clamp t in place to >= 1e-8 (the reference's LearnedTimeDiffusion)."""
    if x.shape[-1] != 64 or evecs.shape[-1] != 64:
        raise _lib.PoseKernError("spectral diffusion kernel is built for C_width = k_eig = 64")
    if clamp_t and not t.is_contiguous():
        raise _lib.PoseKernError("spectral_diffusion: clamp_t needs the parameter's own contiguous storage")
    return _SpectralDiffusion.apply(x, mass.contiguous(), evals.contiguous(), evecs.contiguous(),
                                    t if clamp_t else t.contiguous(), bool(clamp_t))


# ------------------------------------------------------------------------------ H9 fmap solve


class _FmapSolve(torch.autograd.Function):
    """C[b, i, :] = (AAt_b + lambda diag(D_b[i])) ^-1 (BAt_b)[i, :]  (pk_fmap_solve[_backward])."""

    @staticmethod
    def forward(ctx, AAt, BAt, D, lambda_):
        AAt, BAt, D = AAt.contiguous(), BAt.contiguous(), D.contiguous()
        B, K, _ = AAt.shape
        C = torch.empty_like(BAt)
        call("pk_fmap_solve", ptr(AAt), ptr(BAt), ptr(D), float(lambda_), B, K, ptr(C), _lib.stream(AAt.device))
        ctx.save_for_backward(AAt, BAt, D)
        ctx.lambda_ = float(lambda_)
        return C

    @staticmethod
    def backward(ctx, G):
        AAt, BAt, D = ctx.saved_tensors
        G = G.contiguous()
        B, K, _ = AAt.shape
        dBAt = torch.empty_like(BAt)
        part = torch.empty((B, K, K, K), dtype=torch.float32, device=AAt.device)
        call("pk_fmap_solve_backward", ptr(AAt), ptr(BAt), ptr(D), ctx.lambda_, B, K, ptr(G), ptr(dBAt), ptr(part),
             _lib.stream(AAt.device))
        return part.sum(1), dBAt, None, None


def resolvent_mask(evals1: torch.Tensor, evals2: torch.Tensor, gamma: float = 0.5) -> torch.Tensor:
    """get_mask for every crop in one launch (pk_resolvent_mask): evals [B, >=K] (K = the
    mask size = evals1.shape[1] unless sliced views are passed) -> D f32 [B, K, K]."""
    B, K = evals1.shape
    if evals1.stride(1) != 1 or evals2.stride(1) != 1:
        evals1, evals2 = evals1.contiguous(), evals2.contiguous()
    D = torch.empty((B, K, K), dtype=torch.float32, device=evals1.device)
    import ctypes
    call("pk_resolvent_mask", ctypes.c_void_p(evals1.data_ptr()), int(evals1.stride(0)),
         ctypes.c_void_p(evals2.data_ptr()), int(evals2.stride(0)), B, K, float(gamma), ptr(D),
         _lib.stream(evals1.device))
    return D


class _FmapHeadFn(torch.autograd.Function):
    """RegularizedFMNet.forward's batched branch (modeling/dpfm.py:154-195) from the refined
    features to C: pk_fmap_head_fwd (projections, AAt, BAt, the resolvent mask) + pk_fmap_solve;
    backward pk_fmap_solve_backward + pk_fmap_head_bwd, whose expansion writes the feature
    gradients in the features' own storage order."""

    @staticmethod
    def forward(ctx, fx, fy, evecs_x, evecs_y, mass_x, mass_y, evals_x, evals_y, lambda_, gamma):
        import ctypes
        B, N1, Cf = fx.shape
        N2 = fy.shape[1]
        dev = fx.device
        K = 30
        st = lambda t: (ctypes.c_int64 * 3)(*t.stride())  # noqa: E731
        A = torch.empty((B, K, Cf), dtype=torch.float32, device=dev)
        Bm = torch.empty_like(A)
        AAt = torch.empty((B, K, K), dtype=torch.float32, device=dev)
        BAt = torch.empty_like(AAt)
        D = torch.empty_like(AAt)
        wl = int(_lib.lib().pk_fmap_head_work_len(B, int(N1), int(N2)))
        work = torch.empty((max(wl, 1),), dtype=torch.float32, device=dev)
        call("pk_fmap_head_fwd", ptr(evecs_x), int(evecs_x.shape[-1]), ptr(mass_x), ctypes.c_void_p(fx.data_ptr()),
             st(fx), int(N1), ptr(evecs_y), int(evecs_y.shape[-1]), ptr(mass_y), ctypes.c_void_p(fy.data_ptr()),
             st(fy), int(N2), ctypes.c_void_p(evals_x.data_ptr()), int(evals_x.stride(0)),
             ctypes.c_void_p(evals_y.data_ptr()), int(evals_y.stride(0)), B, K, Cf, float(gamma), ptr(A), ptr(Bm),
             ptr(AAt), ptr(BAt), ptr(D), ptr(work), wl, _lib.stream(dev), work=None)
        Cm = torch.empty_like(BAt)
        call("pk_fmap_solve", ptr(AAt), ptr(BAt), ptr(D), float(lambda_), B, K, ptr(Cm), _lib.stream(dev))
        ctx.save_for_backward(evecs_x, evecs_y, mass_x, mass_y, A, Bm, AAt, BAt, D)
        ctx.lambda_ = float(lambda_)
        ctx.fshape = (tuple(fx.shape), tuple(fx.stride()), tuple(fy.shape), tuple(fy.stride()))
        return Cm

    @staticmethod
    def backward(ctx, G):
        import ctypes
        evecs_x, evecs_y, mass_x, mass_y, A, Bm, AAt, BAt, D = ctx.saved_tensors
        G = G.contiguous()
        B, K, _ = AAt.shape
        dev = G.device
        dBAt = torch.empty_like(BAt)
        part = torch.empty((B, K, K, K), dtype=torch.float32, device=dev)
        call("pk_fmap_solve_backward", ptr(AAt), ptr(BAt), ptr(D), ctx.lambda_, B, K, ptr(G), ptr(dBAt), ptr(part),
             _lib.stream(dev))
        (sx, tx, sy, ty) = ctx.fshape
        dfx = torch.empty_strided(sx, tx, dtype=torch.float32, device=dev)  # the features' storage order
        dfy = torch.empty_strided(sy, ty, dtype=torch.float32, device=dev)
        dA, dBm = torch.empty_like(A), torch.empty_like(Bm)
        st = lambda t: (ctypes.c_int64 * 3)(*t.stride())  # noqa: E731
        call("pk_fmap_head_bwd", ptr(part), ptr(dBAt), ptr(A), ptr(Bm), ptr(evecs_x), int(evecs_x.shape[-1]),
             ptr(mass_x), int(sx[1]), ptr(evecs_y), int(evecs_y.shape[-1]), ptr(mass_y), int(sy[1]), B, K, A.shape[2],
             ptr(dA), ptr(dBm), ctypes.c_void_p(dfx.data_ptr()), st(dfx), ctypes.c_void_p(dfy.data_ptr()), st(dfy),
             _lib.stream(dev))
        return dfx, dfy, None, None, None, None, None, None, None, None


def fmap_head(fx, fy, evecs_x, evecs_y, mass_x, mass_y, evals_x, evals_y, lambda_: float, gamma: float):
    """C from the refined features (RegularizedFMNet with evecs_trans = (evecs[..., :30] *
    mass).T), fused: fx [B, N1, 32], fy [B, N2, 32] in rows or channels-first storage."""
    return _FmapHeadFn.apply(fx, fy, evecs_x.contiguous(), evecs_y.contiguous(), mass_x.contiguous(),
                             mass_y.contiguous(), evals_x, evals_y, float(lambda_), float(gamma))


def fmap_solve(AAt: torch.Tensor, BAt: torch.Tensor, D: torch.Tensor, lambda_: float) -> torch.Tensor:
    if AAt.shape[-1] != 30:
        raise _lib.PoseKernError("fmap solve kernel is built for n_fmap = 30")
    return _FmapSolve.apply(AAt, BAt, D, lambda_)


# ------------------------------------------------------------------------------ H8 attention


class _Attention(torch.autograd.Function):
    """softmax(q^T k / sqrt(dim)) v per (crop, head), fused (pk_attention_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, q, k, v):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, D, H, N = q.shape
        M = k.shape[3]
        out = torch.empty_like(q)
        lse = torch.empty((B, H, N, 2), dtype=torch.float32, device=q.device)  # (row max, 1/sum)
        call("pk_attention_fwd", ptr(q), ptr(k), ptr(v), B, D, H, N, M, 0, 0, ptr(out), ptr(lse),
             _lib.stream(q.device), work=("mfma", 2 * 2 * N * M * D * B * H))  # S = Q K^T, O = P V
        ctx.save_for_backward(q, k, v, out, lse)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dout = dout.contiguous()
        B, D, H, N = q.shape
        M = k.shape[3]
        work = attention_bwd_work(B, D, H, N, M, q.device)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        call("pk_attention_bwd", ptr(q), ptr(k), ptr(v), ptr(out), ptr(dout), ptr(lse), B, D, H, N, M, 0, 0,
             ptr(work), ptr(dq), ptr(dk), ptr(dv), 0, 0, _lib.stream(q.device),
             work=("mfma", 5 * 2 * N * M * D * B * H))  # S, dP, dV, dK, dQ: each contraction once
        return dq, dk, dv


def attention_bwd_work(B: int, D: int, H: int, N: int, M: int, device) -> Optional[torch.Tensor]:
    """Scratch of pk_attention_bwd (the dQ partials of key blocks 1 ..; None when one block covers M)."""
    nbytes = int(_lib.lib().pk_attention_bwd_work_size(B, D, H, N, M))
    return torch.empty((nbytes // 4,), dtype=torch.float32, device=device) if nbytes > 0 else None


def attention(query: torch.Tensor, key: torch.Tensor, value: torch.Tensor) -> torch.Tensor:
    """softmax(q^T k / sqrt(d)) v for [B, d, heads, N] fp32 tensors (modeling/dpfm.py:29-37),
    fused in HIP (pk_attention_fwd/_bwd); the score matrix never reaches HBM."""
    if query.shape[1] != 16:
        raise _lib.PoseKernError("attention kernel is built for dim = 16 (gnn_dim 32, 2 heads)")
    if query.dtype != torch.float32:
        raise _lib.PoseKernError("attention kernel computes in fp32")
    return _Attention.apply(query, key, value)


# ------------------------------------------------------------------------------ per-point layers


def linear_wgrad(x: torch.Tensor, dy: torch.Tensor, channels_first: bool, want_bias: bool = True,
                 dw: Optional[torch.Tensor] = None, db: Optional[torch.Tensor] = None, accumulate: bool = False):
    """(dW [O, I], db [O] or None) of y = W x + b over every point (pk_linear_wgrad).
    channels_first=False: x [..., I], dy [..., O]; True: x [B, I, N], dy [B, O, N].
    `dw` / `db` (contiguous, O*I / O elements) are written in place when given, and added
    to when `accumulate` (a weight used by several calls of one forward)."""
    x, dy = x.contiguous(), dy.contiguous()
    if channels_first:
        Bn, I, N = x.shape
        O = dy.shape[1]
        R, layout = Bn * N, 1
    else:
        I, O = x.shape[-1], dy.shape[-1]
        R, N, layout = x.numel() // I, 0, 0
    dev = x.device
    S = (R + 127) // 128
    work = torch.empty((max(S, 1) * (O * I + O),), dtype=torch.float32, device=dev)
    if dw is None:
        dw = torch.empty((O, I), dtype=torch.float32, device=dev)
    if db is None and want_bias:
        db = torch.empty((O,), dtype=torch.float32, device=dev)
    if dw.numel() != O * I or not dw.is_contiguous() or (db is not None and (db.numel() != O or not db.is_contiguous())):
        raise _lib.PoseKernError("linear_wgrad: output buffers must be contiguous [O, I] / [O]")
    call("pk_linear_wgrad", ptr(x), ptr(dy), layout, int(R), I, O, int(N), ptr(work), ptr(dw),
         ptr(db if want_bias else None), int(accumulate), _lib.stream(dev),
         work=("mfma", 2 * int(R) * I * O))
    return dw, db


def linear_wgrad_grouped(calls) -> None:
    """pk_linear_wgrad_grouped: weight / bias gradients of many per-point layers in two
    launches. calls: list of (x, dy, channels_first, dw, db_or_None, accumulate) with dw / db
    contiguous output buffers; a call with accumulate=True adds to the buffers of the one
    earlier call naming the same dw. Inputs must stay alive until the launches complete
    (stream order), as for any stream-ordered op."""
    if not calls:
        return
    arr = (_lib.WgradCall * len(calls))()
    flops = 0
    keep = []
    for k, (x, dy, cf, dw, db, acc) in enumerate(calls):
        sx = sdy = 0
        if (cf and x.dim() == 3 and x.stride(2) == 1 and x.stride(1) == x.shape[2] and x.stride(0) % 4 == 0
                and x.stride(0) >= x.shape[1] * x.shape[2]):  # (stride 0 = an expanded batch: copy)
            sx = x.stride(0)  # a channel slice of a wider channels-first buffer: read in place
        else:
            x = x.contiguous()
        if (cf and dy.dim() == 3 and dy.stride(2) == 1 and dy.stride(1) == dy.shape[2] and dy.stride(0) % 4 == 0
                and dy.stride(0) >= dy.shape[1] * dy.shape[2]):
            sdy = dy.stride(0)
        else:
            dy = dy.contiguous()
        keep += [x, dy]
        if cf:
            Bn, I, N = x.shape
            O, R, layout = dy.shape[1], Bn * N, 1
        else:
            I, O = x.shape[-1], dy.shape[-1]
            R, N, layout = x.numel() // I, 0, 0
        if dw.numel() != O * I or not dw.is_contiguous() or (db is not None and (db.numel() != O or not db.is_contiguous())):
            raise _lib.PoseKernError("linear_wgrad_grouped: output buffers must be contiguous [O, I] / [O]")
        arr[k] = _lib.WgradCall(_dp(x), _dp(dy), ptr(dw).value, ptr(db).value if db is not None else None,
                                int(R), I, O, int(N), layout, int(bool(acc)), 0, int(sx), int(sdy))
        flops += 2 * int(R) * I * O
    n_work = _lib.lib().pk_linear_wgrad_grouped_work(arr, len(calls))
    if n_work < 0:
        raise _lib.PoseKernError("linear_wgrad_grouped: invalid call list")
    dev = calls[0][0].device
    work = torch.empty((max(int(n_work), 1),), dtype=torch.float32, device=dev)
    call("pk_linear_wgrad_grouped", arr, len(calls), ptr(work), int(n_work), _lib.stream(dev),
         work=("mfma", flops))
    # the work buffer and any contiguous() copies are freed on this stream after the launches
    # (the caching allocator reuses them only for later work on the same stream)
    del keep


def clip_rmsprop(params, grads, square_avg, steps, max_norm: float, lr: float, alpha: float, eps: float,
                 norm_out: Optional[torch.Tensor] = None) -> None:
    """clip_grad_norm_(max_norm) + RMSprop step (no momentum / centering / weight decay) over
    lists of f32 device tensors, in two launches (pk_clip_rmsprop). Updates params, grads
    (clipped), square_avg and steps in place."""
    import ctypes
    n = len(params)
    if not (len(grads) == len(square_avg) == n and (steps is None or len(steps) == n)):
        raise _lib.PoseKernError("clip_rmsprop: list lengths differ")
    for t in list(params) + list(grads) + list(square_avg):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise _lib.PoseKernError("clip_rmsprop: f32 contiguous tensors only")
    P = ctypes.c_void_p * n
    arr = lambda ts: P(*[ptr(t).value for t in ts])  # noqa: E731
    numel = (ctypes.c_int64 * n)(*[t.numel() for t in params])
    dev = params[0].device
    work = torch.empty((64,), dtype=torch.float32, device=dev)
    call("pk_clip_rmsprop", arr(params), arr(grads), arr(square_avg), arr(steps) if steps is not None else None,
         numel, n, float(max_norm), float(lr), float(alpha), float(1.0 - alpha), float(eps), ptr(work),
         ptr(norm_out), _lib.stream(dev), work=None)


class _InstNormReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eps):
        B, C, N = x.shape
        y = torch.empty_like(x)
        mean = torch.empty((B * C,), dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        call("pk_instnorm_relu_fwd", ptr(x), B * C, N, float(eps), ptr(y), ptr(mean), ptr(invstd),
             _lib.stream(x.device), work=("hbm", 8 * B * C * N))
        ctx.save_for_backward(x, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, invstd = ctx.saved_tensors
        B, C, N = x.shape
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        call("pk_instnorm_relu_bwd", ptr(x), ptr(dy), ptr(mean), ptr(invstd), B * C, N, ptr(dx),
             _lib.stream(x.device), work=("hbm", 12 * B * C * N))
        return dx, None


def instnorm_relu(x: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """relu(InstanceNorm1d(C, affine=False, eps)(x)) for channels-first f32 x [B, C, N], fused
    forward and backward (pk_instnorm_relu_fwd/_bwd)."""
    if x.dim() != 3 or x.dtype != torch.float32:
        raise _lib.PoseKernError("instnorm_relu takes f32 [B, C, N]")
    return _InstNormReLU.apply(x.contiguous(), eps)


class _WBCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p12, p21, t12, t21, want):
        B, N1 = p12.shape
        N2 = p21.shape[1]
        loss = torch.empty((2, B), dtype=torch.float32, device=p12.device)
        g12 = torch.empty_like(p12) if want else None
        g21 = torch.empty_like(p21) if want else None
        call("pk_wbce", ptr(p12), ptr(t12), N1, ptr(p21), ptr(t21), N2, B, ptr(loss), ptr(g12), ptr(g21),
             _lib.stream(p12.device), work=None)
        ctx.save_for_backward(g12, g21)
        return loss

    @staticmethod
    def backward(ctx, gl):
        g12, g21 = ctx.saved_tensors
        return g12 * gl[0][:, None], g21 * gl[1][:, None], None, None, None


def weighted_bce_pair(p12: torch.Tensor, p21: torch.Tensor, t12: torch.Tensor, t21: torch.Tensor) -> torch.Tensor:
    """Upstream WeightedBCELoss for both overlap directions of every crop (pk_wbce): p f32
    [B, N], t 0/1 masks [B, N] -> loss f32 [2, B] (row 0: p12, row 1: p21)."""
    def mask(t):
        return (t if t.dtype == torch.int8 else (t >= 0.5).to(torch.int8)).contiguous()
    want = torch.is_grad_enabled() and (p12.requires_grad or p21.requires_grad)
    return _WBCE.apply(p12.contiguous(), p21.contiguous(), mask(t12), mask(t21), want)


def _l2_layout(x: torch.Tensor):
    """(tensor, strides) with unit stride on the channel or the point dim (copy otherwise)."""
    import ctypes
    if x.stride(-1) != 1 and x.stride(1) != 1:
        x = x.contiguous()
    return x, (ctypes.c_int64 * 3)(*x.stride())


class _L2Normalize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        B, N, C = x.shape
        y = torch.empty_strided(x.shape, x.stride(), dtype=x.dtype, device=x.device)
        nrm = torch.empty((B * N,), dtype=torch.float32, device=x.device)
        _, st = _l2_layout(x)
        call("pk_l2_normalize_fwd", ctypes_ptr(x), st, B, N, C, ctypes_ptr(y), ptr(nrm), None, _lib.stream(x.device),
             work=("hbm", 8 * B * N * C))
        ctx.save_for_backward(y, nrm)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, nrm = ctx.saved_tensors
        B, N, C = y.shape
        if dy.stride() != y.stride():
            dy = torch.empty_strided(y.shape, y.stride(), dtype=dy.dtype, device=dy.device).copy_(dy)
        dx = torch.empty_strided(y.shape, y.stride(), dtype=y.dtype, device=y.device)
        _, st = _l2_layout(y)
        call("pk_l2_normalize_bwd", ctypes_ptr(y), ctypes_ptr(dy), ptr(nrm), st, B, N, C, ctypes_ptr(dx), None,
             _lib.stream(y.device), work=("hbm", 12 * B * N * C))
        return dx


def ctypes_ptr(t: torch.Tensor):
    """Device pointer of a (possibly non-contiguous, strides passed separately) tensor."""
    import ctypes
    if not t.is_cuda:
        raise _lib.PoseKernError("posekern ops take HIP device tensors only (no CPU fallback)")
    return ctypes.c_void_p(t.data_ptr())


class _L2NormalizeTwo(torch.autograd.Function):
    """F.normalize(x, dim=-1) returned twice: in x's storage order and as a rows [B, N, C]
    copy (one launch); the backward takes both incoming gradients in one launch."""

    @staticmethod
    def forward(ctx, x):
        B, N, C = x.shape
        y = torch.empty_strided(x.shape, x.stride(), dtype=x.dtype, device=x.device)
        y_rows = torch.empty((B, N, C), dtype=x.dtype, device=x.device)
        nrm = torch.empty((B * N,), dtype=torch.float32, device=x.device)
        _, st = _l2_layout(x)
        call("pk_l2_normalize_fwd", ctypes_ptr(x), st, B, N, C, ctypes_ptr(y), ptr(nrm), ptr(y_rows),
             _lib.stream(x.device), work=("hbm", 12 * B * N * C))
        ctx.save_for_backward(y, nrm)
        return y, y_rows

    @staticmethod
    def backward(ctx, dy, dy_rows):
        y, nrm = ctx.saved_tensors
        B, N, C = y.shape
        if dy is not None and dy.stride() != y.stride():
            dy = torch.empty_strided(y.shape, y.stride(), dtype=dy.dtype, device=dy.device).copy_(dy)
        if dy_rows is not None:
            dy_rows = dy_rows.contiguous()
        dx = torch.empty_strided(y.shape, y.stride(), dtype=y.dtype, device=y.device)
        _, st = _l2_layout(y)
        call("pk_l2_normalize_bwd", ctypes_ptr(y), ctypes_ptr(dy) if dy is not None else None, ptr(nrm), st, B, N, C,
             ctypes_ptr(dx), ptr(dy_rows), _lib.stream(y.device), work=("hbm", 16 * B * N * C))
        return dx


def l2_normalize_two(x: torch.Tensor):
    """(F.normalize(x, dim=-1) in x's storage order, the same as a contiguous rows copy)."""
    if x.dim() != 3 or x.dtype != torch.float32:
        raise _lib.PoseKernError("l2_normalize takes f32 [B, N, C]")
    x, _ = _l2_layout(x)
    return _L2NormalizeTwo.apply(x)


def l2_normalize(x: torch.Tensor) -> torch.Tensor:
    """F.normalize(x, p=2, dim=-1) for f32 [B, N, C] in rows or channels-first storage, fused
    forward and backward (pk_l2_normalize_fwd/_bwd); the output keeps x's storage order."""
    if x.dim() != 3 or x.dtype != torch.float32:
        raise _lib.PoseKernError("l2_normalize takes f32 [B, N, C]")
    x, _ = _l2_layout(x)
    return _L2Normalize.apply(x)


def _ovh_args(fx, fy, w0, b0, w1, b1):
    import ctypes
    a = _lib.OverlapHeadArgs()
    for s, f in enumerate((fx, fy)):
        a.x[s] = f.data_ptr()
        for j in range(3):
            a.strides[s][j] = f.stride(j)
        a.N[s] = f.shape[1]
    a.B = fx.shape[0]
    a.w0, a.b0, a.w1, a.b1 = w0.data_ptr(), b0.data_ptr(), w1.data_ptr(), b1.data_ptr()
    return a, ctypes


def _ovh_forward(fx, fy, w0, b0, w1, b1, want: bool):
    """pk_overlap_head_fwd on both shapes: ((s_x, s_y, nrows_x, nrows_y), the saved tensors)."""
    B = fx.shape[0]
    dev = fx.device
    a, ctypes = _ovh_args(fx, fy, w0, b0, w1, b1)
    outs = []
    for s, f in enumerate((fx, fy)):
        N = f.shape[1]
        n = torch.empty_strided(f.shape, f.stride(), dtype=torch.float32, device=dev)
        nrm = torch.empty((B * N,), dtype=torch.float32, device=dev)
        nrows = torch.empty((B, N, 32), dtype=torch.float32, device=dev) if want else None
        h = torch.empty((B, N, 32), dtype=torch.float32, device=dev) if want else None
        sc = torch.empty((B, N), dtype=torch.float32, device=dev)
        a.n[s], a.nrm[s] = n.data_ptr(), nrm.data_ptr()
        a.nrows[s] = nrows.data_ptr() if nrows is not None else None
        a.h[s] = h.data_ptr() if h is not None else None
        a.s[s] = sc.data_ptr()
        outs.append((n, nrm, nrows, h, sc))
    call("pk_overlap_head_fwd", ctypes.addressof(a), _lib.stream(dev),
         work=("hbm", 4 * B * (fx.shape[1] + fy.shape[1]) * (32 + 32 + (64 if want else 0) + 2)))
    (nx, nrx, rx, hx, sx), (ny, nry, ry, hy, sy) = outs
    return (sx, sy, rx, ry), (nx, nrx, rx, hx, sx, ny, nry, ry, hy, sy)


def _ovh_backward(saved, params, dsx, dsy, drx, dry, dadd=(None, None)):
    """pk_overlap_head_bwd on both shapes: (d f_x, d f_y (+ dadd, another consumer's gradient of
    the features, added in the launch), the four weight gradients (None where the grouped launch
    takes them))."""
    from . import layers
    nx, nrx, rx, hx, sx, ny, nry, ry, hy, sy = saved
    w0, b0, w1, b1 = params
    dev = nx.device
    a, ctypes = _ovh_args(nx, ny, w0, b0, w1, b1)
    B = nx.shape[0]
    res = []
    for s, (n, nrm, rows, h, sc, ds, dr, da) in enumerate(((nx, nrx, rx, hx, sx, dsx, drx, dadd[0]),
                                                           (ny, nry, ry, hy, sy, dsy, dry, dadd[1]))):
        N = n.shape[1]
        ds = torch.zeros((B, N), dtype=torch.float32, device=dev) if ds is None else ds.contiguous()
        dr = dr.contiguous() if dr is not None else None
        g = torch.empty((B, N, 1), dtype=torch.float32, device=dev)
        dh = torch.empty((B, N, 32), dtype=torch.float32, device=dev)
        dx = torch.empty_strided(n.shape, n.stride(), dtype=torch.float32, device=dev)
        if da is not None and da.stride() != n.stride():
            da = torch.empty_strided(n.shape, n.stride(), dtype=torch.float32, device=dev).copy_(da)
        a.n[s], a.nrm[s], a.h[s], a.s[s] = n.data_ptr(), nrm.data_ptr(), h.data_ptr(), sc.data_ptr()
        a.ds[s], a.dnr[s] = ds.data_ptr(), (dr.data_ptr() if dr is not None else None)
        a.g[s], a.dh[s], a.dx[s] = g.data_ptr(), dh.data_ptr(), dx.data_ptr()
        a.dadd[s] = da.data_ptr() if da is not None else None
        res.append((rows, h, g, dh, dx, ds, dr, da))
    call("pk_overlap_head_bwd", ctypes.addressof(a), _lib.stream(dev),
         work=("hbm", 4 * B * (nx.shape[1] + ny.shape[1]) * (32 * 5 + 4) +
               sum(4 * d.numel() for d in dadd if d is not None)))
    gw0 = gb0 = gw1 = gb1 = None
    side0 = layers._side_owns(w0, b0)
    side1 = layers._side_owns(w1, b1)
    for rows, h, g, dh, _, _, _, _ in res:
        if side1:
            layers._SIDE.launch(h, g, w1, b1, channels_first=False)
        else:
            dw, db = linear_wgrad(h, g, channels_first=False, want_bias=True)
            gw1 = dw.view(w1.shape) if gw1 is None else gw1 + dw.view(w1.shape)
            gb1 = db if gb1 is None else gb1 + db
        if side0:
            layers._SIDE.launch(rows, dh, w0, b0, channels_first=False)
        else:
            dw, db = linear_wgrad(rows, dh, channels_first=False, want_bias=True)
            gw0 = dw.view(w0.shape) if gw0 is None else gw0 + dw.view(w0.shape)
            gb0 = db if gb0 is None else gb0 + db
    return res[0][4], res[1][4], gw0, gb0, gw1, gb1


class _OverlapHeadFn(torch.autograd.Function):
    """OverlapPredictorNet (modeling/dpfm.py:125-145) for both shapes as one autograd node:
    F.normalize -> Linear(32, 32) + ReLU -> Linear(32, 1) + Sigmoid in one launch per direction
    (pk_overlap_head_fwd / _bwd, bit-identical to the per-layer path). Outputs the two score maps
    and the rows copies of the normalized features (the NCE term's input, utils/loss.py:23-24);
    the weight gradients go to the grouped launch (layers.GroupedWgrad) or are computed here."""

    @staticmethod
    def forward(ctx, fx, fy, w0, b0, w1, b1):
        outs, saved = _ovh_forward(fx, fy, w0, b0, w1, b1, any(ctx.needs_input_grad))
        ctx.params = (w0, b0, w1, b1)
        ctx.save_for_backward(*saved)
        return outs

    @staticmethod
    def backward(ctx, dsx, dsy, drx, dry):
        return _ovh_backward(ctx.saved_tensors, ctx.params, dsx, dsy, drx, dry)


class _LastLinOverlapFn(torch.autograd.Function):
    """The refinement's last_lin on both shapes (modeling/dpfm.py:111-112, desc.transpose(1, 2)
    read in place: channels-first in and out) and the overlap head on its outputs (:125-145) as
    one node, so the two consumers of the refined features — the overlap head and the fmap head
    (models/dpfm.py:80-90) — meet inside it: the fmap head's gradient enters
    pk_overlap_head_bwd's dadd and the features' total gradient leaves that launch (no autograd
    accumulation kernel), then last_lin's input gradient and grouped weight gradient."""

    @staticmethod
    def forward(ctx, d0, d1, wl, bl, w0, b0, w1, b1):
        w2 = wl.view(wl.shape[0], -1)
        Co, Ci = w2.shape
        ys = [torch.empty((d.shape[0], Co, d.shape[2]), dtype=torch.float32, device=d.device) for d in (d0, d1)]
        linear_ex2(*[a for d, y in zip((d0, d1), ys)
                     for a in ((d, w2, bl, 1, d.shape[0] * d.shape[2], d.shape[2], Ci, Co, y), {})])
        fx, fy = ys[0].transpose(1, 2), ys[1].transpose(1, 2)
        want = any(ctx.needs_input_grad)
        (sx, sy, rx, ry), saved = _ovh_forward(fx, fy, w0, b0, w1, b1, want)
        ctx.params = (w0, b0, w1, b1)
        ctx.lin = (wl, bl)
        ctx.save_for_backward(d0, d1, wl, *saved)
        return ys[0], ys[1], sx, sy, rx, ry

    @staticmethod
    def backward(ctx, gy0, gy1, dsx, dsy, drx, dry):
        from . import layers
        sv = ctx.saved_tensors
        d0, d1, wl = sv[:3]
        wl_p, bl = ctx.lin
        w2 = wl.view(wl.shape[0], -1)
        Co, Ci = w2.shape
        dadd = tuple(None if g is None else g.transpose(1, 2) for g in (gy0, gy1))
        dfx, dfy, gw0, gb0, gw1, gb1 = _ovh_backward(sv[3:], ctx.params, dsx, dsy, drx, dry, dadd=dadd)
        dd, gwl, gbl = [torch.empty_like(d0), torch.empty_like(d1)], None, None
        dys = [df.transpose(1, 2) for df in (dfx, dfy)]  # [B, Co, N] contiguous (y's storage)
        linear_ex2(*[a for d, dy, o in zip((d0, d1), dys, dd)
                     for a in ((dy, w2, None, 1, d.shape[0] * d.shape[2], d.shape[2], Co, Ci, o), dict(transw=True))])
        # weight gradients: shape 1 first, the order autograd ran the two last_lin calls' backward in
        for s, (d, dy) in reversed(list(enumerate(zip((d0, d1), dys)))):
            if layers._side_owns(wl_p, bl):
                layers._SIDE.launch(d, dy, wl_p, bl, channels_first=True)
            else:
                dw, db = linear_wgrad(d, dy, channels_first=True, want_bias=bl is not None)
                gwl = dw.view(wl.shape) if gwl is None else gwl + dw.view(wl.shape)
                gbl = db if gbl is None else (gbl + db if db is not None else gbl)
        return dd[0], dd[1], gwl, gbl, gw0, gb0, gw1, gb1


def lastlin_overlap_head(d0: torch.Tensor, d1: torch.Tensor, wl, bl, w0, b0, w1, b1):
    """(y0, y1 [B, 32, N] channels-first last_lin outputs, s_x, s_y, nrows_x, nrows_y): the
    refinement's last_lin + overlap head node (_LastLinOverlapFn)."""
    return _LastLinOverlapFn.apply(d0, d1, wl, bl, w0.contiguous(), b0.contiguous(), w1.contiguous(), b1.contiguous())


def overlap_head(fx: torch.Tensor, fy: torch.Tensor, w0, b0, w1, b1):
    """(s_x [B, N1], s_y [B, N2], nrows_x, nrows_y) of OverlapPredictorNet's score net applied to
    F.normalize(f, dim=-1) of both shapes, f32 [B, N, 32] in rows or channels-first storage."""
    if (fx.dim() != 3 or fy.dim() != 3 or fx.shape[-1] != 32 or fy.shape[-1] != 32 or fx.shape[0] != fy.shape[0]
            or fx.dtype != torch.float32 or fy.dtype != torch.float32):
        raise _lib.PoseKernError("overlap_head takes f32 [B, N, 32] features of both shapes")
    fx, _ = _l2_layout(fx)
    fy, _ = _l2_layout(fy)
    w0, b0, w1, b1 = (t.contiguous() for t in (w0, b0, w1, b1))
    return _OverlapHeadFn.apply(fx, fy, w0, b0, w1, b1)


def mlp3_fwd(x_in: torch.Tensor, x_diff: torch.Tensor, w1, b1, w2, b2, w3, b3):
    """pk_mlp3_fwd: (cat, h1, h2, y) of the DiffusionNet block MLP with its residual."""
    x_in, x_diff = x_in.contiguous(), x_diff.contiguous()
    C = x_in.shape[-1]
    R = x_in.numel() // C
    lead = x_in.shape[:-1]
    dev = x_in.device
    cat = torch.empty(lead + (2 * C,), dtype=torch.float32, device=dev)
    h1 = torch.empty(lead + (C,), dtype=torch.float32, device=dev)
    h2 = torch.empty_like(h1)
    y = torch.empty_like(h1)
    byts = 4 * R * (2 * C + 2 * C + 3 * C + C)  # reads x_in, x_diff (+x_in again), writes cat, h1, h2, y
    call("pk_mlp3_fwd", ptr(x_in), ptr(x_diff), ptr(w1.contiguous()), ptr(b1), ptr(w2.contiguous()), ptr(b2),
         ptr(w3.contiguous()), ptr(b3), int(R), int(C), ptr(cat), ptr(h1), ptr(h2), ptr(y), _lib.stream(dev),
         work=("hbm", byts, 2 * R * C * (2 * C + C + C)))
    return cat, h1, h2, y


def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], channels_first: bool,
               transw: bool = False, relu: bool = False, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """pk_linear_fwd: y = x W^T (+ b) over every point (W [Cout, Cin], or W^T read from a
    [Cin, Cout] tensor when transw). channels_first=False: x [..., Cin] -> [..., Cout];
    True: x [B, Cin, N] -> [B, Cout, N]."""
    x = x.contiguous()
    w = w.contiguous()
    Cout, Cin = (w.shape[1], w.shape[0]) if transw else (w.shape[0], w.shape[1])
    if channels_first:
        Bn, C, N = x.shape
        R, layout = Bn * N, 1
        y = torch.empty((Bn, Cout, N), dtype=x.dtype, device=x.device)
    else:
        C, N, layout = x.shape[-1], 0, 0
        R = x.numel() // max(C, 1)
        y = torch.empty(x.shape[:-1] + (Cout,), dtype=x.dtype, device=x.device)
    assert C == Cin, (C, Cin)
    # a point moves 4 (Cin + Cout) bytes for 2 Cin Cout flops: <= 21 flop/B for these layers,
    # at or below the f32 MFMA ridge (157.3 TFLOP/s / 8 TB/s = 19.7): HBM-bound (flops beside)
    if mask is not None and (mask.shape != y.shape or not mask.is_contiguous()):
        raise _lib.PoseKernError("linear_fwd: mask must be contiguous and shaped like the output")
    # through pk_linear_ex (pk_linear_fwd's own body): every per-point layer launch of the step is
    # then one entry point, so the bench's per-entry timing and the PMC pass's per-kernel bytes
    # describe the same launches
    linear_ex(x, w, bias, layout, int(R), int(N), int(Cin), int(Cout), y, transw=transw, relu=relu, mask=mask)
    return y


def _dp(t: Optional[torch.Tensor]) -> Optional[int]:
    """Device address of a (possibly strided) tensor view, or None."""
    if t is None:
        return None
    if not t.is_cuda:
        raise _lib.PoseKernError("posekern ops take HIP device tensors only (no CPU fallback)")
    return t.data_ptr()


def _linear_args(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], layout: int, R: int, N: int,
                 Cin: int, Cout: int, y: torch.Tensor, ldx: int = 0, ldy: int = 0, transw: bool = False,
                 relu: bool = False, mask: Optional[torch.Tensor] = None, y2: Optional[torch.Tensor] = None,
                 split: int = 0, ldy2: int = 0, store_cf: bool = False, add: Optional[torch.Tensor] = None,
                 lda: int = 0, add_cols: int = 0, act: Optional[int] = None, pre: Optional[torch.Tensor] = None,
                 pre_out: Optional[torch.Tensor] = None, w2: Optional[torch.Tensor] = None,
                 bias2: Optional[torch.Tensor] = None, wsplit: int = 0, add2: Optional[torch.Tensor] = None,
                 lda2: int = 0):
    """(pk_linear_args, algorithmic bytes, flops) of one per-point layer call."""
    w = w.contiguous()
    w2c = w2.contiguous() if w2 is not None else None
    a = _lib.LinearArgs(x=_dp(x), w=_dp(w), bias=_dp(bias), layout=int(layout), N=int(N), R=int(R),
                        Cin=int(Cin), Cout=int(Cout), transw=int(transw), act=int(relu) if act is None else int(act),
                        mask=_dp(mask),
                        ldx=int(ldx), y=_dp(y), ldy=int(ldy), y2=_dp(y2), ldy2=int(ldy2), split=int(split),
                        store_cf=int(store_cf), add=_dp(add), lda=int(lda), add_cols=int(add_cols), pre=_dp(pre),
                        pre_out=_dp(pre_out), w2=_dp(w2c), bias2=_dp(bias2),
                        wsplit=int(wsplit), add2=_dp(add2), lda2=int(lda2))
    # algorithmic bytes: the input rows, the output rows, the weight, and every epilogue /
    # prologue operand the fused launch must move (the ReLU-backward mask, the residual rows, the
    # sigmoid-backward input and its scaled copy) — each crosses HBM exactly once
    byts = 4 * int(R) * (Cin + Cout) + 4 * Cin * Cout
    if mask is not None:
        byts += 4 * int(R) * Cout
    if add is not None:
        byts += 4 * int(R) * (int(add_cols) or Cout)
    if pre is not None:
        byts += 4 * int(R) * Cin * (2 if pre_out is not None else 1)
    if add2 is not None:
        byts += 4 * int(R) * Cout
    return a, (w, w2c), byts, 2 * int(R) * Cin * Cout


def linear_ex(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], layout: int, R: int, N: int,
              Cin: int, Cout: int, y: torch.Tensor, **kw) -> None:
    """pk_linear_ex: a per-point layer writing into caller-placed (strided) outputs with a
    residual / accumulation epilogue. x, y, y2, add are the first elements of their (possibly
    strided) operands; strides as in include/posekern.h (0 = contiguous)."""
    import ctypes
    a, keep, byts, flops = _linear_args(x, w, bias, layout, R, N, Cin, Cout, y, **kw)
    call("pk_linear_ex", ctypes.addressof(a), _lib.stream(x.device), work=("hbm", byts, flops))


def linear_ex2(args0: tuple, kw0: dict, args1: tuple, kw1: dict) -> None:
    """pk_linear_ex2: two independent linear_ex calls (positional args, keyword args each), one
    launch when both are channels-first 32/64-channel layers."""
    import ctypes
    a0, k0, b0, f0 = _linear_args(*args0, **kw0)
    a1, k1, b1, f1 = _linear_args(*args1, **kw1)
    call("pk_linear_ex2", ctypes.addressof(a0), ctypes.addressof(a1), _lib.stream(args0[0].device),
         work=("hbm", b0 + b1, f0 + f1))


def spectral_raw(x: torch.Tensor, ld_in: int, mass, evals, evecs, t, clamp_t: bool, mode: int, out: torch.Tensor,
                 ld_out: int, saved=None, gt=None, accumulate: bool = False, want_raw: bool = True):
    """pk_spectral_diffusion on caller-placed rows (row strides ld_in / ld_out): returns the
    spectral coefficients (mode 0, for the backward) or None."""
    B, N = mass.shape[0], mass.shape[1]
    K = evecs.shape[-1]
    dev = mass.device
    S = (N + 63) // 64
    work = torch.empty((B, S, K, 64), dtype=torch.float32, device=dev)
    scaled = torch.empty((B, K, 64), dtype=torch.float32, device=dev)
    raw = torch.empty((B, K, 64), dtype=torch.float32, device=dev) if (mode == 0 and want_raw) else None
    call("pk_spectral_diffusion", _dp(x), int(ld_in), ptr(mass), ptr(evecs), ptr(evals), ptr(t), int(clamp_t), B, N,
         K, 64, int(mode), ptr(work), ptr(raw), ptr(scaled), ptr(saved), ptr(gt), _dp(out), int(ld_out),
         int(accumulate), _lib.stream(dev), work=("hbm", 16 * B * N * 64))
    return raw


# ------------------------------------------------------------------------------ H10-H13, H15


FD_MODES = {"fp32": 0, "bf16": 1, "bf16x3": 2}


def feat_dist_topk(evecs_x: torch.Tensor, C: torch.Tensor, evecs_y: torch.Tensor, n1: torch.Tensor,
                   n2: torch.Tensor, topk: int, want_dist: bool = False, precision: str = "fp32",
                   work: Optional[torch.Tensor] = None):
    """Nearest CAD rows of every crop point in the spectral embedding (pk_feat_dist_topk).
    evecs_x [B,V1,K>=30], C [B,30,30], evecs_y [B,V2,K>=30], n1/n2 int32 [B].
    precision: "fp32" (the parity path: torch.cdist's augmented contraction on the f32 MFMA),
    "bf16" or "bf16x3" (opt-in: bf16 MFMA cross term, f32 norms). work: optional caller scratch
    (uint8, any contents: the library keeps nothing in it across calls); default: a temporary
    from torch's allocator (none for the one-launch fp32 argmin at full-chip batch sizes)."""
    B, V1, ldx = evecs_x.shape
    _, V2, ldy = evecs_y.shape
    dev = evecs_x.device
    mode = FD_MODES[precision]
    nbytes = int(_lib.lib().pk_feat_dist_work_size(B, V1, V2, int(topk), mode))
    if nbytes < 0:
        raise _lib.PoseKernError("feat_dist_topk: invalid shape / topk / precision")
    if work is None:
        work = torch.empty((max(nbytes, 1),), dtype=torch.uint8, device=dev)
    elif work.numel() < nbytes:
        raise _lib.PoseKernError(f"feat_dist_topk: work holds {work.numel()} bytes, {nbytes} needed")
    idx = torch.empty((B, V2, topk), dtype=torch.int64, device=dev)
    dist = torch.empty((B, V2, topk), dtype=torch.float32, device=dev) if want_dist else None
    call("pk_feat_dist_topk", ptr(evecs_x.contiguous()), ldx, ptr(C.contiguous()), ptr(evecs_y.contiguous()), ldy,
         ptr(n1), ptr(n2), B, V1, V2, int(topk), mode, ptr(work), nbytes, ptr(idx), ptr(dist), _lib.stream(dev),
         work=("mfma" if mode == 0 else "mfma_bf16", 2 * B * V1 * V2 * 32))
    return idx, dist


def nce_select(counts: torch.Tensor, cap: int, num: int, seed: int, ctr: torch.Tensor):
    """pk_nce_select: rows int64 [B, k], valid bool [B, k], k = min(num, cap); advances ctr."""
    B = counts.shape[0]
    k = min(int(num), int(cap))
    dev = counts.device
    rows = torch.empty((B, k), dtype=torch.int64, device=dev)
    valid = torch.empty((B, k), dtype=torch.bool, device=dev)
    call("pk_nce_select", ptr(counts), B, int(cap), int(num), ctypes_u64(seed), ptr(ctr), ptr(rows), ptr(valid),
         _lib.stream(dev))
    return rows, valid


class _NCELoss(torch.autograd.Function):
    """Per-crop NCE loss [B] with gradients computed in the forward pass (pk_nce_loss):
    the backward only scales them by the incoming per-crop gradient."""

    @staticmethod
    def forward(ctx, f1, f2, pairs, rows, valid, nce_t, want):
        B, N1, C = f1.shape
        N2 = f2.shape[1]
        S = rows.shape[1]
        dev = f1.device
        import ctypes
        f1c, f2c = f1.detach(), f2.detach()
        if f1c.stride(-1) != 1 and f1c.stride(1) != 1:  # neither rows nor channels-first storage
            f1c = f1c.contiguous()
        if f2c.stride(-1) != 1 and f2c.stride(1) != 1:
            f2c = f2c.contiguous()
        st = lambda t: (ctypes.c_int64 * 3)(*t.stride())  # noqa: E731
        lse = torch.empty((B, max(S, 1)), dtype=torch.float32, device=dev)
        term = torch.empty_like(lse)
        loss = torch.empty((B,), dtype=torch.float32, device=dev)
        g1 = torch.empty((B, N1, C), dtype=torch.float32, device=dev) if want else None
        g2 = torch.empty((B, N2, C), dtype=torch.float32, device=dev) if want else None
        dxr = torch.empty((2, B, max(S, 1), C), dtype=torch.float32, device=dev) if want else None
        call("pk_nce_loss", ctypes.c_void_p(f1c.data_ptr()), st(f1c), ctypes.c_void_p(f2c.data_ptr()), st(f2c), B, int(N1), int(N2), int(C), ptr(pairs), int(pairs.shape[1]),
             ptr(rows), ptr(valid), int(S), float(nce_t), 0, ptr(lse), ptr(term), ptr(loss), ptr(g1), ptr(g2),
             ptr(dxr), _lib.stream(dev), work=None)
        ctx.save_for_backward(g1, g2)
        return loss

    @staticmethod
    def backward(ctx, gl):
        g1, g2 = ctx.saved_tensors
        s = gl.reshape(-1, 1, 1)
        return (g1 * s if ctx.needs_input_grad[0] else None, g2 * s if ctx.needs_input_grad[1] else None,
                None, None, None, None, None)


def nce_loss(f1: torch.Tensor, f2: torch.Tensor, pairs: torch.Tensor, rows: torch.Tensor, valid: torch.Tensor,
             nce_t: float) -> torch.Tensor:
    """utils/loss.py:17-40 for every crop at once: f1 [B, N1, 32], f2 [B, N2, 32], pairs int64
    [B, cap, 2], rows int64 / valid bool [B, S <= 512] from nce_select -> loss f32 [B]."""
    if f1.dtype != torch.float32 or f1.shape[-1] != 32:
        raise _lib.PoseKernError("pk_nce_loss takes f32 features of width 32")
    want = torch.is_grad_enabled() and (f1.requires_grad or f2.requires_grad)  # (forward runs under no_grad)
    return _NCELoss.apply(f1, f2, pairs.contiguous(), rows.contiguous(), valid.contiguous().view(torch.uint8), nce_t,
                          want)


def affine_cat(a: torch.Tensor, b: torch.Tensor, sub: float, div: float) -> torch.Tensor:
    """cat(((a - sub) / div, (b - sub) / div), 0) with torch's GPU rounding (a product with the
    f32 reciprocal of the scalar divisor), one launch (pk_affine_cat). No gradient: the
    inputs are data (vertex coordinates)."""
    a, b = a.detach().contiguous(), b.detach().contiguous()
    if a.dtype != torch.float32 or b.dtype != torch.float32 or a.shape[1:] != b.shape[1:]:
        raise _lib.PoseKernError("affine_cat: f32 tensors of equal trailing shape")
    out = torch.empty((a.shape[0] + b.shape[0],) + tuple(a.shape[1:]), dtype=torch.float32, device=a.device)
    mul = float(np.float32(1.0) / np.float32(div))
    call("pk_affine_cat", ptr(a), a.numel(), ptr(b), b.numel(), float(sub), mul, ptr(out), _lib.stream(a.device))
    return out


def _nce_raw(f1, f2, pairs, rows, valid, nce_t, want, prenorm=False):
    """pk_nce_loss: (loss [B], g1, g2) with g the gradients of each crop's loss (None unless
    want); prenorm: f1 / f2 already normalized, g with respect to them."""
    import ctypes
    B, N1, C = f1.shape
    N2 = f2.shape[1]
    S = rows.shape[1]
    dev = f1.device
    f1c, f2c = f1.detach(), f2.detach()
    if f1c.stride(-1) != 1 and f1c.stride(1) != 1:
        f1c = f1c.contiguous()
    if f2c.stride(-1) != 1 and f2c.stride(1) != 1:
        f2c = f2c.contiguous()
    st = lambda t: (ctypes.c_int64 * 3)(*t.stride())  # noqa: E731
    lse = torch.empty((B, max(S, 1)), dtype=torch.float32, device=dev)
    term = torch.empty_like(lse)
    loss = torch.empty((B,), dtype=torch.float32, device=dev)
    g1 = torch.empty((B, N1, C), dtype=torch.float32, device=dev) if want else None
    g2 = torch.empty((B, N2, C), dtype=torch.float32, device=dev) if want else None
    dxr = torch.empty((2, B, max(S, 1), C), dtype=torch.float32, device=dev) if want else None
    call("pk_nce_loss", ctypes.c_void_p(f1c.data_ptr()), st(f1c), ctypes.c_void_p(f2c.data_ptr()), st(f2c), B,
         int(N1), int(N2), int(C), ptr(pairs), int(pairs.shape[1]), ptr(rows), ptr(valid), int(S), float(nce_t),
         int(prenorm), ptr(lse), ptr(term), ptr(loss), ptr(g1), ptr(g2), ptr(dxr), _lib.stream(dev), work=None)
    return loss, g1, g2


class _DPFMLossFn(torch.autograd.Function):
    """DPFMLoss.forward (utils/loss.py:44-99) as one autograd node: NCE (pk_nce_loss) and WBCE
    (pk_wbce) with their input gradients, the scalar head (pk_loss_head: Frobenius term,
    weights, sums, dloss/dC12); the backward is one grouped scale (pk_loss_scale)."""

    @staticmethod
    def forward(ctx, C12, f1, f2, o12, o21, C_gt, pairs, rows, valid, t12, t21, w, nce_t, prenorm):
        w_fmap, w_acc, w_nce = w
        want = any(ctx.needs_input_grad[:5])
        B, K = C12.shape[0], C12.shape[1]
        dev = C12.device
        nce, g1, g2 = _nce_raw(f1, f2, pairs, rows, valid, nce_t, want, prenorm)
        N1, N2 = o12.shape[1], o21.shape[1]
        wb = torch.empty((2, B), dtype=torch.float32, device=dev)
        g12 = torch.empty_like(o12) if want else None
        g21 = torch.empty_like(o21) if want else None
        call("pk_wbce", ptr(o12), ptr(t12), N1, ptr(o21), ptr(t21), N2, B, ptr(wb), ptr(g12), ptr(g21),
             _lib.stream(dev), work=None)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        logs = torch.empty((3,), dtype=torch.float32, device=dev)
        dC = torch.empty_like(C12)
        call("pk_loss_head", ptr(C12), ptr(C_gt), B, K, ptr(nce), ptr(wb), float(w_fmap), float(w_acc), float(w_nce),
             ptr(loss), ptr(logs), ptr(dC), _lib.stream(dev), work=None)
        ctx.save_for_backward(dC, g1, g2, g12, g21)
        ctx.scales = (1.0, w_nce / B, w_nce / B, w_acc / B, w_acc / B)
        ctx.mark_non_differentiable(logs)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for `logs` (a fill launch per step)
        return loss, logs

    @staticmethod
    def backward(ctx, gl, _glogs):
        import ctypes
        saved = ctx.saved_tensors
        if gl is None:  # (not materialised: nothing flows into the loss)
            return (None,) * 14
        need = ctx.needs_input_grad[:5]
        outs = [torch.empty_like(t) if (n and t is not None) else None for t, n in zip(saved, need)]
        sel = [i for i, o in enumerate(outs) if o is not None]
        if sel:
            P = ctypes.c_void_p * len(sel)
            call("pk_loss_scale", P(*[saved[i].data_ptr() for i in sel]), P(*[outs[i].data_ptr() for i in sel]),
                 (ctypes.c_int64 * len(sel))(*[saved[i].numel() for i in sel]),
                 (ctypes.c_float * len(sel))(*[ctx.scales[i] for i in sel]), len(sel), ptr(gl.contiguous()),
                 _lib.stream(gl.device), work=None)
        return (*outs, None, None, None, None, None, None, None, None, None)


def dpfm_loss(C12, C_gt, f1, f2, pairs, rows, valid, o12, o21, t12, t21, w_fmap: float, w_acc: float,
              w_nce: float, nce_t: float):
    """DPFMLoss.forward for every crop at once -> (loss 0-d, logs f32 [3] = nce, acc, fmap)."""
    def mask(t):
        return (t if t.dtype == torch.int8 else (t >= 0.5).to(torch.int8)).contiguous()
    if f1.dtype != torch.float32 or f1.shape[-1] != 32:
        raise _lib.PoseKernError("pk_nce_loss takes f32 features of width 32")
    # features whose F.normalize'd rows copy the overlap head already made (l2_normalize_two):
    # the NCE term reads those rows (coalesced) and its gradient joins the overlap head's in
    # the one l2-normalize backward
    n1, n2 = getattr(f1, "_pk_nrows", None), getattr(f2, "_pk_nrows", None)
    prenorm = n1 is not None and n2 is not None
    if prenorm:
        f1, f2 = n1, n2
    return _DPFMLossFn.apply(C12.contiguous(), f1, f2, o12.contiguous(), o21.contiguous(), C_gt.contiguous(),
                             pairs.contiguous(), rows.contiguous(), valid.contiguous().view(torch.uint8),
                             mask(t12), mask(t21), (float(w_fmap), float(w_acc), float(w_nce)), float(nce_t),
                             bool(prenorm))


def rigidity_thresholds(diam: Sequence[float], device) -> torch.Tensor:
    """f32 [B,4]: float32(tau * diam) for tau = 0.3, 0.15, 0.055, 0.065 (Python-float
    products, as the reference compares with `tau * diam_cad`)."""
    rows = [[np.float32(t * float(d)) for t in (0.3, 0.15, 0.055, 0.065)] for d in diam]
    return torch.tensor(np.asarray(rows, dtype=np.float32), device=device)


def rigidity_filter(cand: torch.Tensor, ncand: torch.Tensor, cad: torch.Tensor, pc: torch.Tensor,
                    thr4: torch.Tensor):
    """cand int64 [B,L,2] -> (survivor rows int64 [B,L], count int32 [B])."""
    B, L, _ = cand.shape
    dev = cand.device
    la = torch.zeros((B, L), dtype=torch.int64, device=dev)
    lb = torch.zeros((B, L), dtype=torch.int64, device=dev)  # tail rows stay valid indices (0)
    na = torch.empty((B,), dtype=torch.int32, device=dev)
    nb = torch.empty((B,), dtype=torch.int32, device=dev)
    score = torch.empty((B, L), dtype=torch.float32, device=dev)
    nbytes = int(_lib.lib().pk_rigidity_filter_work_size(B, L, L))
    part = torch.empty((max(nbytes // 4, 1),), dtype=torch.float32, device=dev)
    # f32 VALU work of the first (largest) round: per UNORDERED candidate pair (the term is
    # symmetric) two 3-D distances and |a - b|, ~20 flops (later rounds run on its survivors)
    call("pk_rigidity_filter", ptr(cand.contiguous()), L, ptr(ncand), ptr(cad.contiguous()), cad.shape[1],
         ptr(pc.contiguous()), pc.shape[1], ptr(thr4), B, L, ptr(la), ptr(lb), ptr(na), ptr(nb), ptr(score),
         ptr(part), _lib.stream(dev), work=("valu32", 10 * B * L * L))
    return lb, nb


def inlier_ratio(pairs: torch.Tensor, npairs: torch.Tensor, cad: torch.Tensor, pc_aligned: torch.Tensor,
                 thr: torch.Tensor, layout: int = 0, status: Optional[torch.Tensor] = None,
                 check: Optional[bool] = None) -> torch.Tensor:
    """Per-crop inlier ratio (pk_inlier_ratio). status int32 [B] (optional): per crop 1 when a
    correspondence index lies outside cad / pc_aligned (the pair counts as an outlier, nothing is
    read through it); without it the call checks a temporary one (host sync) unless capturing."""
    B = cad.shape[0]
    ldp = pairs.shape[1] if layout in (0, 2) else pairs.shape[2]
    ir = torch.empty((B,), dtype=torch.float32, device=cad.device)
    st, chk = _index_status(B, cad.device, status, check)
    call("pk_inlier_ratio", ptr(pairs.contiguous()), ldp, int(layout), ptr(npairs), ptr(cad.contiguous()),
         cad.shape[1], ptr(pc_aligned.contiguous()), pc_aligned.shape[1], ptr(thr), B, ptr(ir), ptr(st),
         _lib.stream(cad.device))
    if chk:
        check_index_status(st, "inlier_ratio (correspondence indices)")
    return ir


def mean_f32(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """0-d mean of a float32 device tensor (pk_mean_f32: fixed summation order), into `out` when
    given (a 0-d / 1-element float32 device tensor)."""
    x = x.contiguous()
    if out is None:
        out = torch.empty((), dtype=torch.float32, device=x.device)
    call("pk_mean_f32", ptr(x), x.numel(), ptr(out), _lib.stream(x.device))
    return out


def cgt_lstsq(pairs: torch.Tensor, npairs: torch.Tensor, evecs1: torch.Tensor, evecs2: torch.Tensor,
              cnt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C_from_sparse_P for every crop (pk_cgt_lstsq). cnt int32 [B, ldc] (optional): the pairs per
    crop row among the kept list (ball_query's colcount); without it the call counts them."""
    B, L, _ = pairs.shape
    if cnt is not None:
        assert cnt.dtype == torch.int32 and cnt.dim() == 2 and cnt.shape[0] == B and cnt.is_contiguous()
    out = torch.empty((B, 30, 30), dtype=torch.float32, device=pairs.device)
    nwork = _lib.lib().pk_cgt_lstsq_work_size(L, evecs2.shape[1], B)
    work = torch.empty((nwork,), dtype=torch.float64, device=pairs.device)
    call("pk_cgt_lstsq", ptr(pairs.contiguous()), L, ptr(npairs), ptr(evecs1.contiguous()), evecs1.shape[2],
         evecs1.shape[1], ptr(evecs2.contiguous()), evecs2.shape[2], evecs2.shape[1], B, 30, ptr(cnt),
         int(cnt.shape[1]) if cnt is not None else 0, ptr(work), ptr(out), _lib.stream(pairs.device))
    return out


def ransac(src: torch.Tensor, src_off: torch.Tensor, dst: torch.Tensor, dst_off: torch.Tensor,
           corres: torch.Tensor, cor_off: torch.Tensor, H: int, seed: int = 0, max_dist: float = 0.05,
           hyps: Optional[torch.Tensor] = None, hyp_off: Optional[torch.Tensor] = None,
           nmax: Optional[int] = None, status: Optional[torch.Tensor] = None, check: Optional[bool] = None):
    """Batched RANSAC pose fit (pk_ransac). nmax bounds the correspondences per crop (default:
    all rows of `corres`). status int32 [B] (optional): per crop 1 when a correspondence or
    hypothesis row is out of range (read as row 0 instead); without it the call checks a
    temporary one (host sync) unless capturing. Returns (T f64 [B,4,4], stats f64 [B,3] =
    fitness, rmse, best h)."""
    B = cor_off.numel() - 1
    dev = src.device
    st, chk = _index_status(B, dev, status, check)
    corres = corres.to(torch.int32).contiguous()
    if corres.numel() == 0:  # every crop below ransac_n: keep a valid pointer, kernel returns identity
        corres = torch.zeros((1, 2), dtype=torch.int32, device=dev)
    nmax = int(corres.shape[0]) if nmax is None else int(nmax)
    nbytes = int(_lib.lib().pk_ransac_work_size(B, int(H), nmax))
    work = torch.empty((max(nbytes, 1),), dtype=torch.uint8, device=dev)
    T = torch.empty((B, 4, 4), dtype=torch.float64, device=dev)
    stats = torch.empty((B, 3), dtype=torch.float64, device=dev)
    # fp64 VALU work: ~30 flops per (hypothesis, correspondence) residual + ~6000 per 4-point fit,
    # over the TRUE correspondence counts (nmax is only a capacity): when a probe is timing the
    # launch, the total count is snapshotted on the device and read after the timed region
    wk = None
    if _lib._probe is not None:
        tot = (cor_off[-1] - cor_off[0]).clone()
        wk = lambda: ("valu64", int(H) * (30 * int(tot.item()) + 6000 * B))  # noqa: E731
    call("pk_ransac", ptr(src), ptr(src_off), ptr(dst), ptr(dst_off), ptr(corres),
         ptr(cor_off), ptr(hyps), ptr(hyp_off), ctypes_u64(seed), int(H), float(max_dist), B, nmax, ptr(work),
         nbytes, ptr(T), ptr(stats), ptr(st), _lib.stream(dev), work=wk)
    if chk:
        check_index_status(st, "ransac (correspondence / hypothesis rows)")
    return T, stats


def icp(src: torch.Tensor, src_off: torch.Tensor, tgt: torch.Tensor, tgt_off: torch.Tensor, T_init: torch.Tensor,
        max_dist: float, max_iter: int = 30, rel_fitness: float = 1e-6, rel_rmse: float = 1e-6,
        nsrc_max: Optional[int] = None, ntgt_max: Optional[int] = None, poll: int = 8):
    """Batched point-to-point ICP (pk_icp_init / pk_icp_iterate / pk_icp_result). Iterations are
    enqueued `poll` at a time; between batches the host reads the device count of crops still
    iterating (one 4-byte read). Returns (T f64 [B,4,4], stats f64 [B,4] = fitness, inlier rmse,
    updates, converged)."""
    B = src_off.numel() - 1
    dev = src.device
    if nsrc_max is None:
        nsrc_max = int((src_off[1:] - src_off[:-1]).max()) if B else 0
    if ntgt_max is None:
        ntgt_max = int((tgt_off[1:] - tgt_off[:-1]).max()) if B else 0
    T0 = T_init.to(dtype=torch.float64).reshape(B, 16).contiguous()
    nbytes = int(_lib.lib().pk_icp_work_size(B, int(nsrc_max), int(ntgt_max)))
    work = torch.empty((max(nbytes, 1),), dtype=torch.uint8, device=dev)
    cnt = torch.zeros((1,), dtype=torch.int32, device=dev)
    s = _lib.stream(dev)
    call("pk_icp_init", ptr(src), ptr(src_off), ptr(tgt), ptr(tgt_off), ptr(T0), B, int(nsrc_max), int(ntgt_max),
         ptr(work), nbytes, s)
    done = 0
    while B and done <= max_iter:
        steps = min(int(poll), max_iter + 1 - done)
        call("pk_icp_iterate", ptr(src), ptr(src_off), ptr(tgt), ptr(tgt_off), float(max_dist), int(max_iter),
             float(rel_fitness), float(rel_rmse), B, int(nsrc_max), int(ntgt_max), steps, ptr(work), nbytes,
             ptr(cnt), s, work=("hbm", steps * int(src.shape[0]) * 48))  # upper bound: source + matched target rows
        done += steps
        if int(cnt.item()) == 0:
            break
    T = torch.empty((B, 4, 4), dtype=torch.float64, device=dev)
    stats = torch.empty((B, 4), dtype=torch.float64, device=dev)
    call("pk_icp_result", ptr(work), B, ptr(T), ptr(stats), s)
    return T, stats


def teaser_graph(src: torch.Tensor, dst: torch.Tensor, off: torch.Tensor, nmax: int, beta: float):
    """pk_teaser_graph: the pairwise-consistency bitsets of every crop's matched point pairs ->
    (adj uint64 as int64 [B, nmax, ceil(nmax/64)], deg int32 [B, nmax]) on the device."""
    B = off.numel() - 1
    W = (int(nmax) + 63) // 64
    adj = torch.empty((B, max(int(nmax), 1), max(W, 1)), dtype=torch.int64, device=src.device)
    deg = torch.empty((B, max(int(nmax), 1)), dtype=torch.int32, device=src.device)
    call("pk_teaser_graph", ptr(src), ptr(dst), ptr(off), B, int(nmax), float(beta), ptr(adj), ptr(deg),
         _lib.stream(src.device), work=("valu64", B * int(nmax) * int(nmax) * 20))
    return adj, deg


def teaser_solve_host(src: np.ndarray, dst: np.ndarray, off: np.ndarray, nmax: int, adj: np.ndarray, deg: np.ndarray,
                      params, threads: int = 8):
    """pk_teaser_solve on host arrays (max clique / GNC-TLS / adaptive voting are native host
    code): (T f64 [B,4,4], clique int32 [B, nmax], clique_size int32 [B], info int32 [B, 4])."""
    import ctypes
    B = off.shape[0] - 1
    c = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    src = np.ascontiguousarray(src, dtype=np.float64)
    dst = np.ascontiguousarray(dst, dtype=np.float64)
    off = np.ascontiguousarray(off, dtype=np.int64)
    adj = np.ascontiguousarray(adj)
    deg = np.ascontiguousarray(deg, dtype=np.int32)
    T = np.zeros((B, 4, 4))
    clique = np.zeros((B, max(int(nmax), 1)), dtype=np.int32)
    size = np.zeros(B, dtype=np.int32)
    info = np.zeros((B, 4), dtype=np.int32)
    status = _lib.lib().pk_teaser_solve(c(src), c(dst), c(off), B, int(nmax), c(adj), c(deg), ctypes.byref(params),
                                        int(threads), c(T), c(clique), c(size), c(info))
    if status != 0:
        raise _lib.PoseKernError(f"pk_teaser_solve failed: {_lib._ERRORS.get(status, status)}")
    return T, clique, size, info


def teaser(src: torch.Tensor, dst: torch.Tensor, off: torch.Tensor, nmax: Optional[int] = None,
           noise_bound: float = 0.05, cbar2: float = 1.0, rotation_gnc_factor: float = 1.4,
           rotation_max_iterations: int = 100, rotation_cost_threshold: float = 1e-12,
           kcore_heuristic_threshold: float = 0.5, max_clique_nodes: int = 2_000_000, threads: int = 8):
    """Batched TEASER++ (pk_teaser_graph on the device, one download of the bitsets, then
    pk_teaser_solve on host threads). src / dst f64 [T,3] matched pairs packed by off [B+1]."""
    B = off.numel() - 1
    if nmax is None:
        nmax = int((off[1:] - off[:-1]).max()) if B else 0
    p = _lib.TeaserParams(noise_bound, cbar2, rotation_gnc_factor, rotation_cost_threshold, kcore_heuristic_threshold,
                          int(rotation_max_iterations), 0, int(max_clique_nodes))
    adj, deg = teaser_graph(src, dst, off, nmax, 2.0 * noise_bound * math.sqrt(cbar2))
    return teaser_solve_host(src.cpu().numpy(), dst.cpu().numpy(), off.cpu().numpy(), nmax,
                             adj.cpu().numpy(), deg.cpu().numpy(), p, threads)


def knn(pts: torch.Tensor, off: torch.Tensor, nmax: int, k: int, omit_self: bool = True):
    """pk_knn: (idx int32 [T, k] local to each crop, d2 f64 [T, k]) exact nearest neighbours."""
    T = pts.shape[0]
    idx = torch.empty((max(T, 1), k), dtype=torch.int32, device=pts.device)
    d2 = torch.empty((max(T, 1), k), dtype=torch.float64, device=pts.device)
    B = off.numel() - 1
    call("pk_knn", ptr(pts), ptr(off), B, int(nmax), int(k), int(omit_self), ptr(idx), ptr(d2),
         _lib.stream(pts.device), work=("valu64", B * int(nmax) * int(nmax) * 9))
    return idx[:T], d2[:T]


def pc_local_tri(pts: torch.Tensor, off: torch.Tensor, nmax: int, knn_idx: torch.Tensor):
    """pk_pc_local_tri: (tri int32 [T, k, 2], ntri int32 [T], normals f64 [T, 3])."""
    T, k = knn_idx.shape
    tri = torch.empty((max(T, 1), k, 2), dtype=torch.int32, device=pts.device)
    ntri = torch.empty((max(T, 1),), dtype=torch.int32, device=pts.device)
    nrm = torch.empty((max(T, 1), 3), dtype=torch.float64, device=pts.device)
    call("pk_pc_local_tri", ptr(pts), ptr(off), off.numel() - 1, int(nmax), ptr(knn_idx.contiguous()), int(k), ptr(tri),
         ptr(ntri), ptr(nrm), _lib.stream(pts.device))
    return tri[:T], ntri[:T], nrm[:T]


def soup_triangles(tri: np.ndarray, ntri: np.ndarray) -> np.ndarray:
    """The (center, u, v) soup of one cloud from pc_local_tri's fans (host arrays tri [n, k, 2],
    ntri [n], cloud-local): int32 [sum ntri, 3], point-major, each fan in its stored order."""
    n, k = tri.shape[0], tri.shape[1]
    keep = np.arange(k)[None, :] < ntri[:, None]
    centers = np.broadcast_to(np.arange(n, dtype=np.int32)[:, None], (n, k))[keep]
    return np.ascontiguousarray(np.concatenate([centers[:, None], tri[keep]], axis=1).astype(np.int32))


def tufted_laplacian(pts: np.ndarray, tris: np.ndarray, mollify_factor: float = 1e-5):
    """pk_tufted_laplacian (host): robust_laplacian's mollified tufted-cover intrinsic Delaunay
    Laplacian of one cloud's soup. Returns (i, j, w, mass, nflips): the distinct pairs i < j with
    L_ij = L_ji = -w (L_ii = the sum of the row's w) and the lumped mass, as numpy arrays."""
    pts = np.ascontiguousarray(pts, dtype=np.float64)
    tris = np.ascontiguousarray(tris, dtype=np.int32)
    n, nt = pts.shape[0], tris.shape[0]
    cap = max(3 * nt, 1)
    ii, jj = np.empty(cap, np.int32), np.empty(cap, np.int32)
    ww, mass = np.empty(cap, np.float64), np.empty(max(n, 1), np.float64)
    nnz, nfl = ctypes.c_int64(0), ctypes.c_int64(0)
    call("pk_tufted_laplacian", pts.ctypes.data, n, tris.ctypes.data, nt, float(mollify_factor), cap,
         ii.ctypes.data, jj.ctypes.data, ww.ctypes.data, ctypes.byref(nnz), mass.ctypes.data, ctypes.byref(nfl))
    m = int(nnz.value)
    if m > cap:
        raise _lib.PoseKernError("pk_tufted_laplacian: pair capacity exceeded")
    return ii[:m], jj[:m], ww[:m], mass[:n], int(nfl.value)


def cotan_dense(pts: torch.Tensor, off: torch.Tensor, nmax: int, tri=None, ntri=None, faces=None, foff=None,
                fmax: int = 0, scale: float = 1.0, denom_eps: float = 1e-10):
    """pk_cotan_dense: dense cotan Laplacian f64 [B, nmax, nmax] and lumped mass f64 [B, nmax] of a
    triangle soup (tri / ntri of pc_local_tri) or of mesh faces (int32 [F, 3] packed by foff)."""
    B = off.numel() - 1
    L = torch.empty((B, nmax, nmax), dtype=torch.float64, device=pts.device)
    mass = torch.empty((B, nmax), dtype=torch.float64, device=pts.device)
    k = int(tri.shape[1]) if tri is not None else 0
    call("pk_cotan_dense", ptr(pts), ptr(off), B, int(nmax), ptr(tri), ptr(ntri), k, ptr(faces), ptr(foff), int(fmax),
         float(scale), float(denom_eps), ptr(L), ptr(mass), _lib.stream(pts.device))
    return L, mass


def sym_scale(L: torch.Tensor, off: torch.Tensor, mass: torch.Tensor, eps: float, pad_diag: float) -> torch.Tensor:
    """pk_sym_scale on a copy of L: D^-1/2 (L + eps I) D^-1/2, padding rows / columns -> pad_diag I."""
    A = L.clone()
    B, n, _ = L.shape
    call("pk_sym_scale", ptr(off), B, int(n), float(eps), ptr(mass), float(pad_diag), ptr(A), _lib.stream(L.device))
    return A


def dgemm_cheb(A: torch.Tensor, Y: torch.Tensor, X: Optional[torch.Tensor], alpha: float, beta: float,
               gamma: float) -> torch.Tensor:
    """pk_dgemm_cheb: alpha (A Y) + beta Y + gamma X, batched, fp64."""
    B, n, m = Y.shape
    out = torch.empty_like(Y)
    call("pk_dgemm_cheb", ptr(A), ptr(Y), ptr(X), B, int(n), int(m), float(alpha), float(beta), float(gamma),
         ptr(out), _lib.stream(Y.device), work=("valu64", 2 * B * n * n * m))
    return out


def dgemm_tn(X: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
    """pk_dgemm_tn: X^T Y per crop, fp64 [B, m, m]."""
    B, n, m = X.shape
    G = torch.empty((B, m, m), dtype=torch.float64, device=X.device)
    call("pk_dgemm_tn", ptr(X), ptr(Y), B, int(n), int(m), ptr(G), _lib.stream(X.device))
    return G


def dpotrf(A: torch.Tensor, tau: float = 0.0):
    """pk_dpotrf in place on A [B, n, n] (fp64): lower Cholesky of A + tau I; returns the int32 [B]
    failure flags (device)."""
    B, n, _ = A.shape
    fail = torch.empty((max(B, 1),), dtype=torch.int32, device=A.device)
    call("pk_dpotrf", ptr(A), B, int(n), float(tau), ptr(fail), _lib.stream(A.device),
         work=("valu64", B * n ** 3 // 3))
    return fail[:B]


def dpotrs(L: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """pk_dpotrs: X <- (L L^T)^-1 X in place (X [B, n, m] fp64, contiguous)."""
    B, n, m = X.shape
    call("pk_dpotrs", ptr(L), ptr(X), B, int(n), int(m), _lib.stream(X.device), work=("valu64", 2 * B * n * n * m))
    return X


def icp_fixed(src: torch.Tensor, src_off: torch.Tensor, tgt: torch.Tensor, tgt_off: torch.Tensor,
              T_init: torch.Tensor, max_dist: float, evaluations: int, nsrc_max: int, ntgt_max: int,
              rel_fitness: float = 1e-6, rel_rmse: float = 1e-6):
    """ICP with a fixed number of enqueued evaluations and no host read (HIP-graph capturable):
    max_iteration = evaluations - 1, so every crop stops by the last one (converged crops return
    early in each launch). Same results as `icp` with that max_iteration."""
    B = src_off.numel() - 1
    dev = src.device
    T0 = T_init.to(dtype=torch.float64).reshape(B, 16).contiguous()
    nbytes = int(_lib.lib().pk_icp_work_size(B, int(nsrc_max), int(ntgt_max)))
    work = torch.empty((max(nbytes, 1),), dtype=torch.uint8, device=dev)
    s = _lib.stream(dev)
    call("pk_icp_init", ptr(src), ptr(src_off), ptr(tgt), ptr(tgt_off), ptr(T0), B, int(nsrc_max), int(ntgt_max),
         ptr(work), nbytes, s)
    call("pk_icp_iterate", ptr(src), ptr(src_off), ptr(tgt), ptr(tgt_off), float(max_dist), int(evaluations) - 1,
         float(rel_fitness), float(rel_rmse), B, int(nsrc_max), int(ntgt_max), int(evaluations), ptr(work), nbytes,
         None, s, work=("hbm", int(evaluations) * int(src.shape[0]) * 48))
    T = torch.empty((B, 4, 4), dtype=torch.float64, device=dev)
    stats = torch.empty((B, 4), dtype=torch.float64, device=dev)
    call("pk_icp_result", ptr(work), B, ptr(T), ptr(stats), s)
    return T, stats


def pose_metrics(cad: torch.Tensor, off: torch.Tensor, nmax: int, T_est: torch.Tensor, T_gt: torch.Tensor):
    """pk_pose_metrics -> f64 [B, 7] (ADD, xyz-direction means x3, ADD-S 1-D means x3)."""
    B = off.numel() - 1
    dev = cad.device
    work = torch.empty((13 * B * max(nmax, 1),), dtype=torch.float64, device=dev)
    out = torch.empty((B, 7), dtype=torch.float64, device=dev)
    call("pk_pose_metrics", ptr(cad), ptr(off), B, int(nmax), ptr(T_est.contiguous()), ptr(T_gt.contiguous()),
         ptr(work), ptr(out), _lib.stream(dev))
    return out


def erode_mask(mask: torch.Tensor) -> torch.Tensor:
    F_, H, W = mask.shape
    out = torch.empty_like(mask)
    call("pk_erode_mask", ptr(mask.contiguous()), F_, H, W, ptr(out), _lib.stream(mask.device))
    return out


def sample_rgb(img: torch.Tensor, K: torch.Tensor, pts: torch.Tensor, off: torch.Tensor, nmax: int) -> torch.Tensor:
    """H16: bilinear RGB at the projections of packed camera-frame points -> f32 [T, C]."""
    F_, H, W, C = img.shape
    out = torch.zeros((pts.shape[0], C), dtype=torch.float32, device=img.device)
    call("pk_sample_rgb", ptr(img.contiguous()), F_, H, W, C, ptr(K), ptr(pts), ptr(off), int(nmax), ptr(out),
         _lib.stream(img.device))
    return out


def sample_features(fmap: torch.Tensor, K: torch.Tensor, pts: torch.Tensor, off: torch.Tensor,
                    nmax: int) -> torch.Tensor:
    """H16: bilinear sample of an f32 feature map [F, C, H, W] at the projections of packed
    camera-frame points (grid_sample(align_corners=True, padding_mode="zeros") on pixel
    coordinates) -> f32 [T, C]."""
    if fmap.dtype != torch.float32 or fmap.dim() != 4:
        raise ValueError("sample_features: fmap must be f32 [F, C, H, W]")
    F_, C, H, W = fmap.shape
    out = torch.zeros((pts.shape[0], C), dtype=torch.float32, device=fmap.device)
    call("pk_sample_features", ptr(fmap.contiguous()), F_, C, H, W, ptr(K), ptr(pts), ptr(off), int(nmax), ptr(out),
         _lib.stream(fmap.device))
    return out
