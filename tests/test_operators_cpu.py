"""(f1) Spectral operators, CPU side:
  * the oracle's local fans (scipy Delaunay per neighbourhood) against the half-plane Voronoi rule
    the device kernel uses (restated here in numpy) — pins the kernel's algorithm on the CPU;
  * the Chebyshev-filtered subspace iteration of dpfm_amd.geometry (its block products swapped for
    torch-CPU ones; the kernels themselves are tested in test_operators_gpu.py) against scipy eigsh
    on the oracle's point-cloud Laplacian: eigenvalues, M-orthonormality, residuals.
"""
import numpy as np
import pytest
import torch

from oracle import operators_oracle as OO


def voronoi_fans(pts, nbrs):
    out = set()
    for i in range(pts.shape[0]):
        nb = nbrs[i]
        n = OO.pca_normal(pts, i, nb)
        e1, e2 = OO.tangent_basis(n)
        d = pts[nb] - pts[i]
        q = np.stack([d @ e1, d @ e2], 1)
        for j in range(len(nb)):
            u = np.array([-q[j, 1], q[j, 0]])
            mj = 0.5 * q[j]
            tlo, thi, hl = -np.inf, np.inf, -1
            ok = True
            for l in range(len(nb)):
                if l == j:
                    continue
                s = u @ q[l]
                r = 0.5 * (q[l] @ q[l]) - mj @ q[l]
                if s > 0 and r / s < thi:
                    thi, hl = r / s, l
                elif s < 0 and r / s > tlo:
                    tlo = r / s
                elif s == 0 and r < 0:
                    ok = False
            if ok and tlo < thi and hl >= 0:
                out.add((i, int(nb[j]), int(nb[hl])))
    return out


def ellipsoid(rng, n, axes=(5.0, 4.0, 3.0)):
    u = rng.normal(size=(n, 3))
    return u / np.linalg.norm(u, axis=1, keepdims=True) * np.asarray(axes)


def test_local_fans_voronoi_rule_matches_delaunay():
    rng = np.random.default_rng(0)
    pts = ellipsoid(rng, 300)
    idx, _ = OO.knn(pts, 30)
    ref = {(i, j, l) for (i, j, l) in OO.local_triangles(pts, idx)}
    got = voronoi_fans(pts, idx)
    canon = lambda S: {(i, min(j, l), max(j, l)) for (i, j, l) in S}  # noqa: E731
    assert canon(got) == canon(ref)


def test_subspace_iteration_matches_eigsh(monkeypatch):
    from dpfm_amd import geometry, ops

    def cheb(A, Y, X, alpha, beta, gamma):
        out = alpha * torch.bmm(A, Y) + beta * Y
        return out + gamma * X if X is not None else out

    def potrf(A, tau=0.0):
        L = torch.linalg.cholesky(A + tau * torch.eye(A.shape[-1], dtype=A.dtype))
        A.copy_(L)
        return torch.zeros(A.shape[0], dtype=torch.int32)

    monkeypatch.setattr(ops, "dgemm_cheb", cheb)
    monkeypatch.setattr(ops, "dgemm_tn", lambda X, Y: torch.bmm(X.transpose(1, 2), Y))
    monkeypatch.setattr(ops, "dpotrf", potrf)
    monkeypatch.setattr(ops, "dpotrs", lambda L, X: X.copy_(torch.cholesky_solve(X, torch.tril(L))))
    rng = np.random.default_rng(1)
    shapes = [ellipsoid(rng, 350), ellipsoid(rng, 300, (6.0, 3.0, 2.0))]
    nmax, k, eps = 350, 24, 1e-8
    Ls, Ms = [], []
    for p in shapes:
        idx, _ = OO.knn(p, 30)
        L, M = OO.cotan_laplacian(p, OO.local_triangles(p, idx), scale=1.0 / 3.0, denom_eps=0.0)
        Ls.append(L)
        Ms.append(M)
    A = np.zeros((2, nmax, nmax))
    upper = max(np.abs(L).sum(1).max() / M.min() for L, M in zip(Ls, Ms))
    for b, (L, M) in enumerate(zip(Ls, Ms)):
        n = L.shape[0]
        s = 1.0 / np.sqrt(M)
        A[b, :n, :n] = (L + eps * np.eye(n)) * s[:, None] * s[None, :]
        A[b, n:, n:] = np.eye(nmax - n) * upper
    ev, W, it, res = geometry.subspace_eigs(torch.as_tensor(A), [350, 300], k, tol=1e-9)
    print("iterations", it, "residual", res)
    assert float(res.max()) < 1e-9 and it < 60
    for b, (L, M) in enumerate(zip(Ls, Ms)):
        n = L.shape[0]
        ref, V = OO.eigsh_operators(L, M, k, eps)
        np.testing.assert_allclose(ev[b].numpy(), np.sort(ref), rtol=1e-8, atol=1e-10)
        evecs = W[b, :n].numpy() / np.sqrt(M)[:, None]
        np.testing.assert_allclose(evecs.T @ (M[:, None] * evecs), np.eye(k), atol=1e-8)
        r = (L + eps * np.eye(n)) @ evecs - (M[:, None] * evecs) * ev[b].numpy()[None, :]
        assert np.abs(r).max() < 1e-7


def _tufted_dense(n, i, j, w):
    L = np.zeros((n, n))
    L[i, j] -= w
    L[j, i] -= w
    L[np.arange(n), np.arange(n)] += np.bincount(i, w, n) + np.bincount(j, w, n)
    return L


@pytest.mark.parametrize("n,noise", [(150, 0.02), (400, 0.02), (300, 0.0)])
def test_tufted_laplacian_matches_oracle(n, noise):
    """pk_tufted_laplacian (host C++, robust_laplacian's mollified tufted-cover intrinsic Delaunay
    Laplacian) vs the oracle's restatement on the oracle's fan soup of a (noisy) ellipsoid cloud:
    L within 1e-12 of its scale (the two flip queues run in different orders), mass to 1e-13; the
    flipped operator has no negative edge weight while the soup's has some; flips preserve area."""
    from dpfm_amd import ops
    rng = np.random.default_rng(n)
    s = ellipsoid(rng, n) + noise * rng.normal(size=(n, 3))
    ki, _ = OO.knn(s, 30)
    tris = OO.local_triangles(s, ki)
    Lr, Mr, flips = OO.tufted_laplacian(s, tris)
    i, j, w, m, nf = ops.tufted_laplacian(s, np.asarray(tris, dtype=np.int32))
    assert nf > 0 and flips > 0
    assert np.all(i < j) and np.all(np.diff(i.astype(np.int64) * n + j) > 0)  # distinct, sorted pairs
    L = _tufted_dense(n, i, j, w)
    assert np.abs(L - Lr).max() <= 1e-12 * np.abs(Lr).max()
    np.testing.assert_allclose(m, Mr, rtol=1e-13)
    assert w.min() >= -1e-12 * w.max()
    Ls, Ms = OO.cotan_laplacian(s, tris, scale=1.0 / 3.0, denom_eps=0.0)
    assert (Ls[~np.eye(n, dtype=bool)] > 1e-12 * np.abs(Ls).max()).any()  # the soup had negative weights
    np.testing.assert_allclose(m.sum(), Ms.sum(), rtol=1e-12)


def test_tufted_laplacian_without_flips_is_the_soup():
    """An equilateral planar grid (every angle 60 degrees: Delaunay on the cover, nothing to flip,
    nothing to mollify), each triangle listed three times with mixed orientations as the point-
    cloud soup lists it: exactly the soup cotan Laplacian / 3 (pk_cotan_dense's soup operator)."""
    from dpfm_amd import ops
    nx, ny = 7, 6
    pts = np.array([[x + 0.5 * (y % 2), y * np.sqrt(3) / 2, 0.0] for y in range(ny) for x in range(nx)])
    tris = []
    for y in range(ny - 1):
        for x in range(nx - 1):
            a, b, c, d = y * nx + x, y * nx + x + 1, (y + 1) * nx + x, (y + 1) * nx + x + 1
            t1, t2 = ((a, b, d), (a, d, c)) if y % 2 else ((a, b, c), (b, d, c))
            tris += [t1, (t1[1], t1[2], t1[0]), (t1[0], t1[2], t1[1]), t2, (t2[2], t2[0], t2[1]), (t2[1], t2[0], t2[2])]
    i, j, w, m, nf = ops.tufted_laplacian(pts, np.asarray(tris, dtype=np.int32))
    assert nf == 0
    Ls, Ms = OO.cotan_laplacian(pts, tris, scale=1.0 / 3.0, denom_eps=0.0)
    n = pts.shape[0]
    assert np.abs(_tufted_dense(n, i, j, w) - Ls).max() <= 1e-13 * np.abs(Ls).max()
    np.testing.assert_allclose(m, Ms, rtol=1e-13)
    Lr, Mr, fl = OO.tufted_laplacian(pts, tris)
    assert fl == 0 and np.abs(Lr - Ls).max() <= 1e-13 * np.abs(Ls).max()


def test_tufted_laplacian_mollifies_degenerate_triangles():
    """A soup with a collinear (zero-area) triangle: mollification (1e-5 x the mean edge length)
    makes every cover triangle strictly valid, so the operator is finite; without it the
    degenerate triangle's cotangents are not. Rejects out-of-range / repeated corners."""
    from dpfm_amd import _lib, ops
    pts = np.array([[0.0, 0, 0], [1, 0, 0], [2, 0, 0], [1, 1, 0], [1, -1, 0]])
    tris = np.array([[0, 1, 2], [0, 1, 3], [1, 2, 3], [0, 4, 1], [1, 4, 2]], dtype=np.int32)
    i, j, w, m, _ = ops.tufted_laplacian(pts, tris, 1e-5)
    assert np.isfinite(w).all() and np.isfinite(m).all()
    Lr, Mr, _ = OO.tufted_laplacian(pts, [tuple(t) for t in tris], 1e-5)
    assert np.abs(_tufted_dense(5, i, j, w) - Lr).max() <= 1e-9 * np.abs(Lr).max()
    for bad in ([[0, 1, 5]], [[0, 0, 1]]):
        with pytest.raises(_lib.PoseKernError):
            ops.tufted_laplacian(pts, np.array(bad, dtype=np.int32))
