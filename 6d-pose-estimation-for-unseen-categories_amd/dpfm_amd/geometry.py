"""Spectral operators on the device — the (f1) row of SURVEY.md §8(f).

The reference computes the operators on the CPU when it fills its cache:
  CAD:  dataset/object.py:214 geometry.get_operators(verts, faces, normals, k_eig=64)
        -> potpourri3d cotan_laplacian(denom_eps=1e-10) + vertex_areas (+ 1e-8 * mean)
  crop: dataset/object.py:246 geometry.get_operators(verts, faces=[], k_eig=64)
        -> robust_laplacian.point_cloud_laplacian(verts) (30 neighbours, local Delaunay fans)
  both: scipy eigsh(L + 1e-8 I, k=64, M=diag(mass), sigma=1e-8), evals clipped at 0
(upstream diffusion-net geometry.compute_operators).

Here every step runs in hand-written kernels (csrc/operators.hip): kNN, the local fans, the
cotan assembly, and a shift-invert subspace iteration (eigsh's sigma mode) for the 64 smallest
eigenpairs of A = M^-1/2 (L + eps I) M^-1/2: a blocked fp64 Cholesky of A + tau I (pk_dpotrf),
blocked triangular solves (pk_dpotrs) and the block products pk_dgemm_cheb / pk_dgemm_tn; only the
m x m Rayleigh-Ritz / Cholesky-QR problems (m = 2k) use torch.linalg on the device. (A Chebyshev-filtered
variant, cheb_filter, converges too slowly on crop Laplacians: their spectral bound reaches ~1e4
against lambda_64 ~ 3, because of tiny-mass points.) Dense fp64
operators: N <= ~5000 per shape (200 MB for the CAD), well inside HBM.

Returns what compute_operators returns that the model reads (mass, L, evals, evecs) plus the
tangent frames (build_tangent_frames from the PCA normals of the crop's 30-neighbourhoods, or the
mesh's area-weighted vertex normals); gradX / gradY feed only gradient features, which this model
configuration does not use (models/dpfm.py:22-30, with_gradient_features=False), and are None.
Parity unpinned."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import ops


@dataclass
class SpectralOperators:
    mass: torch.Tensor     # f64 [B, nmax]
    L: torch.Tensor        # f64 [B, nmax, nmax] dense cotan Laplacian
    evals: torch.Tensor    # f64 [B, k]
    evecs: torch.Tensor    # f64 [B, nmax, k], M-orthonormal
    normals: Optional[torch.Tensor]  # f64 [T, 3] (point clouds)
    iterations: int
    residual: torch.Tensor  # f64 [B] max eigen-residual / spectral bound over the k pairs
    frames: Optional[torch.Tensor] = None  # f64 [T, 3, 3] (basisX, basisY, normal) per point
    gradX = None
    gradY = None


def tangent_frames(normals: torch.Tensor) -> torch.Tensor:
    """diffusion-net build_tangent_frames: basisX = the x axis (the y axis where |n . x| >= 0.9)
    projected to the tangent plane and normalized, basisY = n x basisX; [T, 3, 3] rows (X, Y, n)."""
    n = normals
    ex = torch.zeros_like(n)
    ex[:, 0] = 1.0
    ey = torch.zeros_like(n)
    ey[:, 1] = 1.0
    cand = torch.where((n[:, 0].abs() < 0.9)[:, None], ex, ey)
    bx = cand - (cand * n).sum(-1, keepdim=True) * n
    bx = bx / bx.norm(dim=-1, keepdim=True)
    by = torch.cross(n, bx, dim=-1)
    return torch.stack((bx, by, n), dim=-2)


def mesh_vertex_normals(pts: torch.Tensor, faces: torch.Tensor) -> torch.Tensor:
    """diffusion-net mesh_vertex_normals: area-weighted face normals summed per vertex, normalized."""
    a, b, c = pts[faces[:, 0]], pts[faces[:, 1]], pts[faces[:, 2]]
    fn = torch.cross(b - a, c - a, dim=-1)
    vn = torch.zeros_like(pts)
    for k in range(3):
        vn.index_add_(0, faces[:, k].long(), fn)
    return vn / vn.norm(dim=-1, keepdim=True).clamp(min=1e-300)


def _pack(verts: Sequence[np.ndarray], device):
    off = np.concatenate([[0], np.cumsum([v.shape[0] for v in verts])]).astype(np.int64)
    pts = torch.as_tensor(np.concatenate([np.asarray(v, dtype=np.float64) for v in verts]), device=device)
    return pts, torch.as_tensor(off, device=device), int(max(v.shape[0] for v in verts))


def cheb_filter(A, X, degree: int, a: float, b: float, a0: float = 0.0):
    """Scaled Chebyshev filter (Zhou & Saad) damping [a, b], amplifying below a."""
    e, c = (b - a) / 2.0, (b + a) / 2.0
    sigma = e / (a0 - c)
    tau = 2.0 / sigma
    Y = ops.dgemm_cheb(A, X, None, sigma / e, -c * sigma / e, 0.0)
    for _ in range(2, degree + 1):
        s2 = 1.0 / (tau - sigma)
        Y, X = ops.dgemm_cheb(A, Y, X, 2.0 * s2 / e, -2.0 * s2 * c / e, -sigma * s2), Y
        sigma = s2
    return Y


def _orth(X, passes: int = 2):
    """Cholesky QR: X <- X R^-1 with R^T R = X^T X (the m x m Gram from pk_dgemm_tn; the m x m
    Cholesky and triangular solve stay on the device, no host round trip). One pass suffices after
    an inverse application to an orthonormal block (its condition number is at most the subspace's
    eigenvalue spread, ~1e2-1e3, so CholQR loses ~kappa^2 u ~ 1e-10); two for the random start."""
    for _ in range(passes):
        G = ops.dgemm_tn(X, X)
        R = torch.linalg.cholesky(0.5 * (G + G.transpose(1, 2)), upper=True)
        X = torch.linalg.solve_triangular(R, X, upper=True, left=False).contiguous()
    return X


def subspace_eigs(A: torch.Tensor, counts: Sequence[int], k: int, extra: int = 64, tol: float = 1e-8,
                  max_iter: int = 200, seed: int = 0, tau_rel: float = 1e-6, rr_every: int = 3):
    """k smallest eigenpairs of each symmetric A[b] (padding rows / columns of crop b beyond
    counts[b] hold a large diagonal) by shift-invert subspace iteration — eigsh's sigma mode:
    A + tau I = L L^T once (pk_dpotrf; tau escalated x10 when a pivot fails, as compute_operators
    escalates eps), (A + tau I)^-1 = L^-T L^-1 I once (pk_dpotrs with N right-hand sides), then per
    iteration X <- (A + tau I)^-1 X (pk_dgemm_cheb) and one Cholesky-QR pass; every rr_every
    iterations a Rayleigh-Ritz step with A itself (subspace iteration converges without it; it
    extracts the eigenpairs and tests convergence, and its m x m eigensolve is the costly part). Converged when every wanted residual |A x - theta x| <= tol * theta_k
    (ARPACK's relative criterion at the k-th Ritz value; the operators are stored in fp32
    downstream). The rate per iteration is (lambda_k + tau) / (lambda_m + tau), m = k + extra."""
    B, N, _ = A.shape
    m = min(k + extra, min(counts))
    if m < k:
        raise ValueError(f"a shape has fewer points ({min(counts)}) than eigenpairs requested ({k})")
    upper = float(A.abs().sum(-1).amax())  # Gershgorin bound over the batch
    tau = tau_rel * upper
    for _ in range(6):
        Lf = A.clone()
        if not bool(ops.dpotrf(Lf, tau).any()):
            break
        tau *= 10.0
    else:
        raise RuntimeError("failed to compute eigendecomp (shifted Cholesky kept failing)")
    # the shifted inverse once (the factor serves ~30 iterations): two blocked sweeps over the
    # identity with m = N right-hand sides (large, efficient updates), then one dense product per
    # iteration instead of 2 x N / 64 dependent block steps
    Ainv = torch.eye(N, dtype=A.dtype, device=A.device).repeat(B, 1, 1)
    ops.dpotrs(Lf, Ainv)
    del Lf
    rng = np.random.default_rng(seed)
    X0 = rng.standard_normal((B, N, m))
    for b, n in enumerate(counts):
        X0[b, n:] = 0.0
    X = _orth(torch.as_tensor(X0, device=A.device))
    theta, res, it = None, None, 0
    for it in range(1, max_iter + 1):
        X = _orth(ops.dgemm_cheb(Ainv, X, None, 1.0, 0.0, 0.0), passes=1)
        if it % rr_every and it != max_iter:  # Rayleigh-Ritz (and the convergence test) every rr_every
            continue
        AX = ops.dgemm_cheb(A, X, None, 1.0, 0.0, 0.0)
        H = ops.dgemm_tn(X, AX)
        theta, Wt = torch.linalg.eigh(0.5 * (H + H.transpose(1, 2)))  # m x m Rayleigh-Ritz, on the device
        X = torch.bmm(X, Wt)
        AX = torch.bmm(AX, Wt)
        R = AX[:, :, :k] - X[:, :, :k] * theta[:, None, :k]
        res = R.norm(dim=1).amax(-1) / theta[:, k - 1].abs().clamp(min=1e-300)
        if float(res.max()) < tol:
            break
    return theta[:, :k], X[:, :, :k], it, res


def get_operators(verts: Sequence[np.ndarray], faces: Optional[Sequence[np.ndarray]] = None, k_eig: int = 64,
                  n_neighbors: int = 30, eps: float = 1e-8, device=None, **eig_kw) -> SpectralOperators:
    """Operators of a batch of shapes: triangle meshes when `faces` is given (the CAD path), point
    clouds otherwise (the crop path)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    pts, off, nmax = _pack(verts, dev)
    counts = [int(v.shape[0]) for v in verts]
    if faces is None:
        return point_cloud_operators(pts, off, counts, k_eig=k_eig, n_neighbors=n_neighbors, eps=eps, **eig_kw)
    fo = np.concatenate([[0], np.cumsum([f.shape[0] for f in faces])]).astype(np.int64)
    fc = torch.as_tensor(np.concatenate([np.asarray(f, dtype=np.int32) for f in faces]), device=dev)
    L, mass = ops.cotan_dense(pts, off, nmax, faces=fc, foff=torch.as_tensor(fo, device=dev),
                              fmax=int(max(f.shape[0] for f in faces)), scale=1.0, denom_eps=1e-10)
    for b, n in enumerate(counts):  # vertex_areas + eps * mean (compute_operators)
        mass[b, :n] += eps * mass[b, :n].mean()
    return _spectral(pts, off, counts, L, mass, None, k_eig, eps, faces=faces, **eig_kw)


def point_cloud_operators(pts: torch.Tensor, off: torch.Tensor, counts: Sequence[int], k_eig: int = 64,
                          n_neighbors: int = 30, eps: float = 1e-8, robust: bool = True,
                          mollify_factor: float = 1e-5, **eig_kw) -> SpectralOperators:
    """The crop path (dataset/object.py:246 get_operators(verts=pcd_depth, faces=[])) on packed
    device points: f64 [T, 3] rows off[b]..off[b+1] per cloud (e.g. Crops.pc64 / Crops.off as
    CropFormation leaves them). kNN, the local fans and the eigensolver run on the device;
    robust=True (robust_laplacian.point_cloud_laplacian) lifts each cloud's fan soup to its
    mollified tufted cover and flips it to intrinsic Delaunay on the host (pk_tufted_laplacian,
    one thread per cloud), the result scattered back into the dense device L; robust=False keeps
    the soup's own cotan Laplacian (pk_cotan_dense, the same operator before any flip)."""
    pts = pts.to(torch.float64).contiguous()
    off = off.to(device=pts.device, dtype=torch.int64).contiguous()
    counts = [int(c) for c in counts]
    nmax = max(counts)
    idx, _ = ops.knn(pts, off, nmax, n_neighbors, omit_self=True)
    tri, ntri, normals = ops.pc_local_tri(pts, off, nmax, idx)
    if robust:
        L, mass = tufted_dense(pts, off, counts, nmax, tri, ntri, mollify_factor)
    else:
        L, mass = ops.cotan_dense(pts, off, nmax, tri=tri, ntri=ntri, scale=1.0 / 3.0, denom_eps=0.0)
    return _spectral(pts, off, counts, L, mass, normals, k_eig, eps, **eig_kw)


def tufted_dense(pts, off, counts, nmax, tri, ntri, mollify_factor=1e-5):
    """Dense device (L f64 [B, nmax, nmax], mass f64 [B, nmax]) of the clouds' tufted-cover
    Laplacians (pk_tufted_laplacian per cloud on host threads; the distinct pairs scattered with
    index_put_ — no duplicate indices, so the result is deterministic)."""
    from concurrent.futures import ThreadPoolExecutor
    dev = pts.device
    B = len(counts)
    o = off.cpu().numpy()
    P, T, NT = pts.cpu().numpy(), tri.cpu().numpy(), ntri.cpu().numpy()

    def one(b):
        a, e = int(o[b]), int(o[b + 1])
        return ops.tufted_laplacian(P[a:e], ops.soup_triangles(T[a:e], NT[a:e]), mollify_factor)
    with ThreadPoolExecutor(max_workers=max(1, min(B, 16))) as ex:
        res = list(ex.map(one, range(B)))
    L = torch.zeros((B, nmax, nmax), dtype=torch.float64, device=dev)
    mass = torch.zeros((B, nmax), dtype=torch.float64, device=dev)
    for b, (i, j, w, m, _) in enumerate(res):
        n = counts[b]
        diag = np.bincount(i, weights=w, minlength=n) + np.bincount(j, weights=w, minlength=n)
        it, jt = torch.as_tensor(i.astype(np.int64), device=dev), torch.as_tensor(j.astype(np.int64), device=dev)
        wt = torch.as_tensor(-w, device=dev)
        L[b].index_put_((it, jt), wt)
        L[b].index_put_((jt, it), wt)
        L[b, :n, :n].diagonal().copy_(torch.as_tensor(diag, device=dev))
        mass[b, :n] = torch.as_tensor(m, device=dev)
    return L, mass


def _spectral(pts, off, counts, L, mass, normals, k_eig, eps, faces=None, **eig_kw) -> SpectralOperators:
    """eigsh(L + eps I, k, M = diag(mass), sigma) for the assembled operators, then the frames."""
    dev = L.device
    for b, n in enumerate(counts):
        mass[b, n:] = 1.0
    upper = float(L.abs().sum(-1).amax() / mass.amin())
    A = ops.sym_scale(L, off, mass, eps, pad_diag=upper)
    evals, W, iters, res = subspace_eigs(A, counts, k_eig, **eig_kw)
    evecs = W / mass.sqrt()[:, :, None]
    for b, n in enumerate(counts):
        evecs[b, n:] = 0.0
        mass[b, n:] = 0.0
    if normals is None:  # mesh: vertex normals from the faces (crop-local indices -> packed rows)
        fl = torch.cat([torch.as_tensor(np.asarray(f, dtype=np.int64), device=dev) + int(o)
                        for f, o in zip(faces, off[:-1].cpu().tolist())])
        normals = mesh_vertex_normals(pts, fl)
    return SpectralOperators(mass=mass, L=L, evals=evals.clamp(min=0.0), evecs=evecs, normals=normals,
                             iterations=iters, residual=res, frames=tangent_frames(normals))
