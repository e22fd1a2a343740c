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
                      appears up to three times) — the soup operator before robust_laplacian's flips
  tufted_laplacian    robust_laplacian.point_cloud_laplacian's intrinsic stage (Sharp & Crane
                      2020; geometry-central buildTuftedLaplacian): mollified edge lengths, the
                      tufted cover (faces sorted about each edge, facing sides glued), intrinsic
                      Delaunay flips, cotan Laplacian / lumped mass x 1/2 (cover) x 1/3 (soup)
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


def tufted_laplacian(pts: np.ndarray, tris, mollify_factor: float = 1e-5, tol: float = 1e-12):
    """Dense (L, mass, flips) of the soup `tris` (list of (a, b, c), cloud-local) over pts [n, 3]:
    robust_laplacian.point_cloud_laplacian's stage after the local triangulation.
      1. eps = mollify_factor * mean distinct-edge length; every edge length grows by
         delta = max(0, max over triangle corners of l_c - l_a - l_b + eps);
      2. tufted cover: face f -> sides (f, +1) = (a, b, c) and (f, -1) = (a, c, b); around each soup
         edge {u < v} the faces are ordered by the angle of their apex about the axis v - u
         (measured from the first face's apex, ties by face order); the side of face i running
         u -> v is glued to the side of face i + 1 (cyclically) running v -> u;
      3. intrinsic flips of every edge with cot(alpha) + cot(beta) < -2 tol until none is left
         (flipped lengths from the planar layout of the two triangles);
      4. L = sum over cover edges of w (e_i - e_j)(e_i - e_j)^T, w = (cot alpha + cot beta) / 2,
         mass = area / 3 per corner, both x 1/6. Parity unpinned (robust_laplacian is absent)."""
    import math
    from collections import deque
    n = pts.shape[0]
    tris = [tuple(int(x) for x in t) for t in tris]
    dist = lambda u, v: float(np.sqrt(((pts[u] - pts[v]) ** 2).sum()))  # noqa: E731
    soup_len, fins = {}, {}
    for f, t in enumerate(tris):
        for r in range(3):
            u, v = t[r], t[(r + 1) % 3]
            key = (min(u, v), max(u, v))
            if key not in soup_len:
                soup_len[key] = dist(u, v)
                fins[key] = []
            fins[key].append((f, r))
    mean = sum(soup_len.values()) / len(soup_len)
    if mollify_factor > 0:
        eps, delta = mollify_factor * mean, 0.0
        for t in tris:
            ls = [soup_len[(min(t[r], t[(r + 1) % 3]), max(t[r], t[(r + 1) % 3]))] for r in range(3)]
            for r in range(3):
                delta = max(delta, ls[(r + 2) % 3] - ls[r] - ls[(r + 1) % 3] + eps)
        soup_len = {k: l + delta for k, l in soup_len.items()}
    # cover faces as vertex triples; halfedge (face, corner) runs face[c] -> face[c + 1]
    faces = []
    for (a, b, c) in tris:
        faces.append([a, b, c])
        faces.append([a, c, b])
    twin, elen, eof = {}, [], {}

    def side(f, r, tail):  # halfedge of face f's soup corner r in the side whose tail is `tail`
        a, b = tris[f][r], tris[f][(r + 1) % 3]
        if tail == a:
            return (2 * f, r)
        back = faces[2 * f + 1]
        for c in range(3):
            if back[c] == b and back[(c + 1) % 3] == a:
                return (2 * f + 1, c)
        raise AssertionError
    for (u, v), lst in fins.items():
        ax = pts[v] - pts[u]
        ax = ax / (np.linalg.norm(ax) or 1.0)
        ref, angs = None, []
        for (f, r) in lst:
            w = tris[f][(r + 2) % 3]
            p = pts[w] - pts[u]
            p = p - (p @ ax) * ax
            if ref is None and np.linalg.norm(p) > 0:
                e1 = p / np.linalg.norm(p)
                ref = (e1, np.cross(ax, e1))
            th = math.atan2(p @ ref[1], p @ ref[0]) if ref is not None else 0.0
            angs.append(th + 2 * math.pi if th < 0 else th)
        order = sorted(range(len(lst)), key=lambda i: angs[i])  # stable: ties keep face order
        m = len(order)
        for q in range(m):
            f, r = lst[order[q]]
            fn, rn = lst[order[(q + 1) % m]]
            A, B = side(f, r, u), side(fn, rn, v)
            twin[A], twin[B] = B, A
            e = len(elen)
            elen.append(soup_len[(u, v)])
            eof[A] = eof[B] = e
    nxt = lambda h: (h[0], (h[1] + 1) % 3)  # noqa: E731
    prv = lambda h: (h[0], (h[1] + 2) % 3)  # noqa: E731
    tail = lambda h: faces[h[0]][h[1]]  # noqa: E731

    def area(a, b, c):
        s = 0.5 * (a + b + c)
        x = s * (s - a) * (s - b) * (s - c)
        return math.sqrt(x) if x > 0 else 0.0

    def cot(h):
        lc, la, lb = elen[eof[h]], elen[eof[nxt(h)]], elen[eof[prv(h)]]
        return (la * la + lb * lb - lc * lc) / (4.0 * area(la, lb, lc))

    def weight(h):
        return 0.5 * (cot(h) + cot(twin[h]))
    edge_he = {}
    for h, e in eof.items():
        edge_he.setdefault(e, h)
    queue, inq, flips = deque(range(len(elen))), set(range(len(elen))), 0
    while queue:
        e = queue.popleft()
        inq.discard(e)
        h = edge_he[e]
        if weight(h) >= -tol:
            continue
        t = twin[h]
        if t[0] == h[0]:
            continue
        a, b, c, d = nxt(h), prv(h), nxt(t), prv(t)  # j->k, k->i, i->l, l->j
        vi, vj, vk, vl = tail(h), tail(t), tail(b), tail(d)
        L0 = elen[e]
        lik, ljk, lil, ljl = elen[eof[b]], elen[eof[a]], elen[eof[c]], elen[eof[d]]
        kx = (L0 * L0 + lik * lik - ljk * ljk) / (2 * L0)
        ky = math.sqrt(max(0.0, lik * lik - kx * kx))
        lx = (L0 * L0 + lil * lil - ljl * ljl) / (2 * L0)
        ly = -math.sqrt(max(0.0, lil * lil - lx * lx))
        # rebuild the two faces: (k, l, j) and (l, k, i); outer halfedges keep their edges
        outer = {a: ((h[0], 2), vj), b: ((t[0], 1), vk), c: ((t[0], 2), vi), d: ((h[0], 1), vl)}
        old = {x: (twin[x], eof[x]) for x in outer}
        faces[h[0]] = [vk, vl, vj]
        faces[t[0]] = [vl, vk, vi]
        for x in outer:
            del twin[x], eof[x]
        nh, nt = (h[0], 0), (t[0], 0)
        twin[nh], twin[nt] = nt, nh
        eof[nh] = eof[nt] = e
        for x, (slot, _) in outer.items():
            tw, ex = old[x]
            eof[slot] = ex
            if tw in outer:
                twin[slot] = outer[tw][0]
            else:
                twin[slot] = tw
                twin[tw] = slot
            edge_he[ex] = slot
            if ex not in inq:
                inq.add(ex)
                queue.append(ex)
        elen[e] = math.hypot(kx - lx, ky - ly)
        edge_he[e] = nh
        flips += 1
    L = np.zeros((n, n))
    mass = np.zeros(n)
    for e, h in edge_he.items():
        i, j = tail(h), tail(twin[h])
        if i == j:
            continue
        w = weight(h) / 6.0
        L[i, j] -= w
        L[j, i] -= w
        L[i, i] += w
        L[j, j] += w
    for f, fc in enumerate(faces):
        A = area(*(elen[eof[(f, r)]] for r in range(3)))
        for v in fc:
            mass[v] += A / 18.0
    return L, mass, flips
