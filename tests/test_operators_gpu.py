"""(f1) Spectral operators on the device (csrc/operators.hip, dpfm_amd/geometry.py) against the
numpy / scipy restatement (oracle/operators_oracle.py):
  * pk_knn: indices and squared distances bit-exact on ragged crops (incl. a crop smaller than k);
  * pk_pc_local_tri: the local Delaunay fans equal the oracle's scipy Delaunay fans (as triangle
    sets), PCA normals equal up to sign;
  * pk_cotan_dense: the soup (1/3-scaled) and mesh-face Laplacians / masses within 1e-12 relative
    (fp64 atomics: the summation order of a shared entry is not fixed);
  * pk_dgemm_cheb / pk_dgemm_tn against torch fp64;
  * get_operators (point clouds — robust_laplacian's tufted-cover intrinsic Delaunay Laplacian —
    and a mesh) against scipy eigsh(L + eps I, k, M, sigma = eps) on the oracle's operator:
    eigenvalues, M-orthonormality, residuals;
  * the new-crop chain (crop formation -> device operators at 2000 points, k = 64 -> DPFMNet ->
    InferStep) against the same oracle per crop and the oracle model on the chained operators.
"""
import numpy as np
import pytest
import torch

from oracle import operators_oracle as OO
from test_operators_cpu import ellipsoid

pytestmark = pytest.mark.gpu


def _pack(shapes, device):
    off = np.concatenate([[0], np.cumsum([s.shape[0] for s in shapes])]).astype(np.int64)
    return (torch.as_tensor(np.concatenate(shapes), device=device), torch.as_tensor(off, device=device),
            max(s.shape[0] for s in shapes))


def _shapes(seed=0):
    rng = np.random.default_rng(seed)
    return [ellipsoid(rng, 400), ellipsoid(rng, 257, (6.0, 2.0, 2.5)), rng.normal(size=(20, 3)),
            ellipsoid(rng, 333, (3.0, 3.0, 3.0))]


def test_knn_bitexact(device):
    from dpfm_amd import ops
    shapes = _shapes()
    pts, off, nmax = _pack(shapes, device)
    idx, d2 = ops.knn(pts, off, nmax, 30)
    idx, d2 = idx.cpu().numpy(), d2.cpu().numpy()
    o = off.cpu().numpy()
    for b, s in enumerate(shapes):
        ri, rd = OO.knn(s, 30)
        kk = min(30, s.shape[0] - 1)
        np.testing.assert_array_equal(idx[o[b]:o[b + 1], :kk], ri[:, :kk])
        np.testing.assert_array_equal(d2[o[b]:o[b + 1], :kk], rd[:, :kk])
        if kk < 30:
            assert (idx[o[b]:o[b + 1], kk:] == -1).all()


def test_local_fans_and_cotan_match_oracle(device):
    from dpfm_amd import ops
    shapes = [s for s in _shapes(1) if s.shape[0] > 100]
    pts, off, nmax = _pack(shapes, device)
    idx, _ = ops.knn(pts, off, nmax, 30)
    tri, ntri, nrm = ops.pc_local_tri(pts, off, nmax, idx)
    L, M = ops.cotan_dense(pts, off, nmax, tri=tri, ntri=ntri, scale=1.0 / 3.0, denom_eps=0.0)
    tri, ntri, nrm, L, M = (x.cpu().numpy() for x in (tri, ntri, nrm, L, M))
    o = off.cpu().numpy()
    canon = lambda S: {(i, min(j, l), max(j, l)) for (i, j, l) in S}  # noqa: E731
    for b, s in enumerate(shapes):
        ki, _ = OO.knn(s, 30)
        ref = OO.local_triangles(s, ki)
        got = [(i, int(tri[o[b] + i, c, 0]), int(tri[o[b] + i, c, 1])) for i in range(s.shape[0])
               for c in range(ntri[o[b] + i])]
        assert canon(got) == canon(ref)
        for i in range(0, s.shape[0], 37):
            nr = OO.pca_normal(s, i, ki[i])
            assert abs(abs(nr @ nrm[o[b] + i]) - 1.0) < 1e-12
        Lr, Mr = OO.cotan_laplacian(s, ref, scale=1.0 / 3.0, denom_eps=0.0)
        n = s.shape[0]
        np.testing.assert_allclose(L[b, :n, :n], Lr, rtol=0, atol=1e-12 * np.abs(Lr).max())
        np.testing.assert_allclose(M[b, :n], Mr, rtol=1e-12)
        assert np.abs(L[b, n:]).max(initial=0) == 0 and np.abs(M[b, n:]).max(initial=0) == 0


def _hull_mesh(rng, n, axes):
    from scipy.spatial import ConvexHull
    v = ellipsoid(rng, n, axes)
    return v, ConvexHull(v).simplices.astype(np.int32)


def test_mesh_cotan_matches_oracle(device):
    from dpfm_amd import ops
    rng = np.random.default_rng(2)
    meshes = [_hull_mesh(rng, 300, (5, 4, 3)), _hull_mesh(rng, 211, (2, 3, 4))]
    pts, off, nmax = _pack([m[0] for m in meshes], device)
    fo = np.concatenate([[0], np.cumsum([m[1].shape[0] for m in meshes])]).astype(np.int64)
    fc = torch.as_tensor(np.concatenate([m[1] for m in meshes]), device=device)
    L, M = ops.cotan_dense(pts, off, nmax, faces=fc, foff=torch.as_tensor(fo, device=device),
                           fmax=int(max(m[1].shape[0] for m in meshes)), scale=1.0, denom_eps=1e-10)
    L, M = L.cpu().numpy(), M.cpu().numpy()
    for b, (v, f) in enumerate(meshes):
        Lr, Mr = OO.cotan_laplacian(v, [tuple(x) for x in f], scale=1.0, denom_eps=1e-10)
        n = v.shape[0]
        np.testing.assert_allclose(L[b, :n, :n], Lr, rtol=0, atol=1e-12 * np.abs(Lr).max())
        np.testing.assert_allclose(M[b, :n], Mr, rtol=1e-12)


def test_dgemm_kernels(device):
    from dpfm_amd import ops
    g = torch.Generator(device="cpu").manual_seed(0)
    A = torch.randn(3, 150, 150, dtype=torch.float64, generator=g)
    A = (A + A.transpose(1, 2)).to(device)
    X = torch.randn(3, 150, 70, dtype=torch.float64, generator=g).to(device)
    Y = torch.randn(3, 150, 70, dtype=torch.float64, generator=g).to(device)
    out = ops.dgemm_cheb(A, Y, X, 0.7, -0.3, 0.25)
    ref = 0.7 * torch.bmm(A, Y) - 0.3 * Y + 0.25 * X
    assert (out - ref).abs().max() < 1e-12 * ref.abs().max()
    G = ops.dgemm_tn(X, Y)
    assert (G - torch.bmm(X.transpose(1, 2), Y)).abs().max() < 1e-12 * G.abs().max()


@pytest.mark.parametrize("kind", ["cloud", "cloud-soup", "mesh"])
def test_get_operators_matches_eigsh(device, kind):
    from dpfm_amd import geometry
    rng = np.random.default_rng(3)
    k, eps = 32, 1e-8
    if kind.startswith("cloud"):
        robust = kind == "cloud"
        shapes = [ellipsoid(rng, 500) + 0.01 * rng.normal(size=(500, 3)), ellipsoid(rng, 420, (6.0, 3.0, 2.0))]
        op = geometry.get_operators(shapes, k_eig=k, device=device, tol=1e-10, robust=robust)
        refs = []
        for b, s in enumerate(shapes):
            ki, _ = OO.knn(s, 30)
            tris = OO.local_triangles(s, ki)
            Lr, Mr = (OO.tufted_laplacian(s, tris)[:2] if robust
                      else OO.cotan_laplacian(s, tris, scale=1.0 / 3.0, denom_eps=0.0))
            n = s.shape[0]
            assert np.abs(op.L[b, :n, :n].cpu().numpy() - Lr).max() <= 1e-10 * np.abs(Lr).max()
            refs.append((Lr, Mr))
    else:
        meshes = [_hull_mesh(rng, 500, (5, 4, 3)), _hull_mesh(rng, 400, (2, 3, 4))]
        shapes = [m[0] for m in meshes]
        op = geometry.get_operators(shapes, faces=[m[1] for m in meshes], k_eig=k, device=device, tol=1e-10)
        refs = []
        for v, f in meshes:
            Lr, Mr = OO.cotan_laplacian(v, [tuple(x) for x in f], scale=1.0, denom_eps=1e-10)
            refs.append((Lr, Mr + eps * Mr.mean()))
    ev, V, M = op.evals.cpu().numpy(), op.evecs.cpu().numpy(), op.mass.cpu().numpy()
    Fr = op.frames.cpu().numpy()  # orthonormal right-handed frames, third row = the normal
    np.testing.assert_allclose(np.einsum("tij,tkj->tik", Fr, Fr), np.broadcast_to(np.eye(3), Fr.shape), atol=1e-12)
    np.testing.assert_allclose(np.linalg.det(Fr), 1.0, atol=1e-12)
    for b, (s, (Lr, Mr)) in enumerate(zip(shapes, refs)):
        n = s.shape[0]
        np.testing.assert_allclose(M[b, :n], Mr, rtol=1e-12)
        er, _ = OO.eigsh_operators(Lr, Mr, k, eps)
        np.testing.assert_allclose(ev[b], np.sort(er), rtol=1e-7, atol=1e-9)
        E = V[b, :n]
        np.testing.assert_allclose(E.T @ (Mr[:, None] * E), np.eye(k), atol=1e-7)
        r = (Lr + eps * np.eye(n)) @ E - (Mr[:, None] * E) * ev[b][None, :]
        assert np.abs(r).max() < 1e-6 * max(1.0, ev[b].max())


@pytest.mark.parametrize("n", [64, 150, 333])
def test_dpotrf_dpotrs(device, n):
    """Blocked Cholesky (64-blocks, ragged last block) and the blocked triangular solves against
    torch fp64; a non-SPD matrix sets the failure flag."""
    from dpfm_amd import ops
    g = torch.Generator(device="cpu").manual_seed(n)
    M = torch.randn(2, n, n, dtype=torch.float64, generator=g)
    A = (M @ M.transpose(1, 2) / n + 0.1 * torch.eye(n, dtype=torch.float64)).to(device)
    Lf = A.clone()
    fail = ops.dpotrf(Lf, 0.05)
    assert not bool(fail.any())
    ref = torch.linalg.cholesky(A.cpu() + 0.05 * torch.eye(n, dtype=torch.float64))
    got = torch.tril(Lf.cpu())
    assert (got - ref).abs().max() < 1e-12 * ref.abs().max()
    X = torch.randn(2, n, 70, dtype=torch.float64, generator=g)
    Y = ops.dpotrs(Lf, X.to(device).contiguous()).cpu()
    Yr = torch.cholesky_solve(X, ref)
    assert (Y - Yr).abs().max() < 1e-10 * Yr.abs().max()
    bad = A.clone()
    bad[1] -= 10.0 * torch.eye(n, dtype=torch.float64, device=device)
    assert ops.dpotrf(bad, 0.0).cpu().tolist() == [0, 1]


def test_new_crop_chain_2000_k64(device):
    """(f1) chained: CropFormation (2 frames, 2000-point crops) -> pipeline.device_crop_operators
    (kNN, local fans, cotan soup, shift-invert eigensolver, k = 64, on the device) -> InferStep.
    Operators per crop vs the oracle's scipy eigsh on the oracle's own tufted-cover Laplacian of the
    same f32-rounded crop points (dataset/object.py:246): L to 1e-10, mass to 1e-12, eigenvalues to 1e-7,
    M-orthonormality and residuals as above; the chain's f32 fields are the f64 result rounded.
    Then the model on the chained operators: C vs the oracle DPFMNet in fp64 within 3x the fp32
    reference's error (as test_configs_gpu's chain test), poses finite."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import InferStep, device_crop_operators, make_frame_batch, model_batch
    from oracle import dpfm_model_oracle as M
    B, N, k, eps = 2, 2000, 64, 1e-8
    fb, op = make_frame_batch(B, 1024, N, seed=41, device=device)
    crops = CropFormation(n1=1024, npoint=N, seed=3)(fb)
    op2 = device_crop_operators(op, crops, k_eig=k, tol=1e-10)
    so = op2.pc_spectral
    counts = crops.n2.cpu().tolist()
    assert min(counts) == N
    off = crops.off.cpu().numpy()
    pts = crops.pc64.float().double().cpu().numpy()
    ev, V, Mm = so.evals.cpu().numpy(), so.evecs.cpu().numpy(), so.mass.cpu().numpy()
    assert torch.equal(op2.pc_evecs[:, :N].cpu(), so.evecs.float().cpu())
    assert torch.equal(op2.pc_mass[:, :N].cpu(), so.mass.float().cpu())
    for b in range(B):
        s = pts[off[b]:off[b + 1]]
        ki, _ = OO.knn(s, 30)
        Lr, Mr, _ = OO.tufted_laplacian(s, OO.local_triangles(s, ki))
        np.testing.assert_allclose(Mm[b, :N], Mr, rtol=1e-12)
        Lg = so.L[b, :N, :N].cpu().numpy()
        assert np.abs(Lg - Lr).max() <= 1e-10 * np.abs(Lr).max()
        er, _ = OO.eigsh_operators(Lr, Mr, k, eps)
        np.testing.assert_allclose(ev[b], np.sort(er), rtol=1e-7, atol=1e-9)
        E = V[b, :N]
        np.testing.assert_allclose(E.T @ (Mr[:, None] * E), np.eye(k), atol=1e-7)
        r = (Lr + eps * np.eye(N)) @ E - (Mr[:, None] * E) * ev[b][None, :]
        assert np.abs(r).max() < 1e-6 * max(1.0, ev[b].max())
    torch.manual_seed(2)
    ref = M.DPFMNet()
    mine = DPFMNet().to(device)
    mine.load_state_dict(ref.state_dict())
    out = InferStep(mine, hypotheses=256, seed=1)(fb, op2, crops)
    torch.cuda.synchronize()
    mb = model_batch(op2, crops)
    cpu = {kk: {a: v.cpu() for a, v in d.items() if a in ("xyz", "mass", "evals", "evecs")} for kk, d in mb.items()}
    with torch.no_grad():
        C32 = ref(cpu)[0]
        truth = M.DPFMNet().double()
        truth.load_state_dict(ref.state_dict())
        C64 = truth({kk: {a: v.double() for a, v in d.items()} for kk, d in cpu.items()})[0]
    e_ref = (C32.double() - C64).abs().max().item()
    assert (out["C"].cpu().double() - C64).abs().max().item() <= 3 * e_ref + 1e-6 * (1 + C64.abs().max().item())
    assert torch.isfinite(out["T"]).all()
