"""(f1) Spectral operators — TEST INFRASTRUCTURE ONLY (tests/ import it; the product never does).

Restates the reference's operator construction (dataset/object.py:214, 246 -> upstream
diffusion-net geometry.compute_operators / get_operators) with numpy /
scipy, parity unpinned (diffusion-net, robust_laplacian and potpourri3d are absent):

  knn                 exact k nearest neighbours, fp64 ((dx dx + dy dy) + dz dz), ties -> lower index
  pca_normal          smallest-eigenvalue direction of the neighbourhood covariance
  local_triangles     robust_laplacian's point-cloud step: per point, the 2-D Delaunay
                      triangulation (scipy / Qhull) of the point and its k neighbours projected
                      on the tangent plane; the triangles incident to the point
  cotan_laplacian     pp3d.cotan_laplacian (denom_eps 1e-10) + vertex areas (area / 3 per corner)
                      for a triangle list; the point-cloud soup is scaled by 1/3 (each triangle
                      appears up to three times), as robust_laplacian does — without its
                      tufted-cover intrinsic-Delaunay flips and mollification
  eigsh_operators     compute_operators' eigsh(L + eps I, k, M = diag(mass), sigma = eps),
                      evals clipped at 0
"""
from __future__ import annotations

import numpy as np


def knn(pts: np.ndarray, k: int, omit_self: bool = True):
    d = pts[:, None, :] - pts[None, :, :]
    d2 = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    if omit_self:
        np.fill_diagonal(d2, np.inf)
    idx = np.argsort(d2, axis=1, kind="stable")[:, :k]
    return idx.astype(np.int32), np.take_along_axis(d2, idx, 1)


def tangent_basis(n: np.ndarray):
    a = np.argmin(np.abs(n))
    e = np.zeros(3)
    e[a] = 1.0
    e1 = np.cross(n, e)
    e1 /= np.linalg.norm(e1)
    return e1, np.cross(n, e1)


def pca_normal(pts: np.ndarray, i: int, nb: np.ndarray) -> np.ndarray:
    P = pts[np.concatenate([[i], nb])]
    c = P - P.mean(0)
    w, v = np.linalg.eigh(c.T @ c)
    n = v[:, 0]
    return n / np.linalg.norm(n)


def local_triangles(pts: np.ndarray, nbrs: np.ndarray) -> list:
    """Triangles (i, j, l) of every point's local Delaunay fan, CCW in its tangent basis."""
    from scipy.spatial import Delaunay
    out = []
    for i in range(pts.shape[0]):
        nb = nbrs[i]
        n = pca_normal(pts, i, nb)
        e1, e2 = tangent_basis(n)
        d = pts[nb] - pts[i]
        q = np.stack([d @ e1, d @ e2], 1)
        tri = Delaunay(np.concatenate([np.zeros((1, 2)), q]))
        for s in tri.simplices:
            if 0 not in s:
                continue
            a, b = [x for x in np.roll(s, -list(s).index(0))[1:]]
            qa, qb = q[a - 1], q[b - 1]
            if qa[0] * qb[1] - qa[1] * qb[0] < 0:  # CCW around the centre
                a, b = b, a
            out.append((i, int(nb[a - 1]), int(nb[b - 1])))
    return out


def cotan_laplacian(pts: np.ndarray, tris, scale: float = 1.0, denom_eps: float = 1e-10):
    n = pts.shape[0]
    L = np.zeros((n, n))
    mass = np.zeros(n)
    for (a, b, c) in tris:
        for (o, u, v) in ((a, b, c), (b, c, a), (c, a, b)):
            eu, ev = pts[u] - pts[o], pts[v] - pts[o]
            cr = np.cross(eu, ev)
            w = 0.5 * (eu @ ev) / (np.linalg.norm(cr) + denom_eps)
            L[u, v] -= w
            L[v, u] -= w
            L[u, u] += w
            L[v, v] += w
        area = 0.5 * np.linalg.norm(np.cross(pts[b] - pts[a], pts[c] - pts[a]))
        mass[[a, b, c]] += area / 3.0
    return L * scale, mass * scale


def eigsh_operators(L: np.ndarray, mass: np.ndarray, k: int, eps: float = 1e-8):
    import scipy.sparse
    import scipy.sparse.linalg as sla
    Ls = scipy.sparse.csc_matrix(L) + scipy.sparse.identity(L.shape[0]) * eps
    evals, evecs = sla.eigsh(Ls, k=k, M=scipy.sparse.diags(mass), sigma=eps)
    return np.clip(evals, 0.0, np.inf), evecs
