"""CPU: the oracle's restatements agree with each other (torch literal vs C vs numpy)."""
import math

import numpy as np
import pytest
import torch

from oracle import dpfm_oracle as O
from _util import c_fps, c_ball_query, boundary_cloud


@pytest.mark.parametrize("n,npoint,dups", [(50, 50, 0), (300, 64, 0), (257, 100, 40), (2345, 2000, 0)])
def test_fps_torch_literal_matches_c(coracle, n, npoint, dups):
    rng = np.random.default_rng(n)
    xyz = (rng.normal(size=(n, 3)) * 7 + np.array([0, 0, 110])).astype(np.float32)
    if dups:  # exact duplicates exercise the first-index tie rule
        xyz[rng.integers(0, n, dups)] = xyz[rng.integers(0, n, dups)]
    start = int(rng.integers(0, n))
    ref = O.farthest_point_sample(torch.from_numpy(xyz).t(), ratio=npoint / n, start=start, npoint=npoint).numpy()
    got = c_fps(coracle, xyz, start, npoint)
    np.testing.assert_array_equal(ref, got)


def test_fps_npoint_rounding():
    # dataset/object.py:146-147: int(2000/N * N) is 1999 for some N (as the published crops show)
    vals = {O.fps_npoint(n) for n in range(2001, 6000)}
    assert vals == {1999, 2000}


def test_torch_sum3_is_left_to_right():
    rng = np.random.default_rng(0)
    a = rng.normal(size=(100000, 3)).astype(np.float32) * 100
    t = torch.sum(torch.from_numpy(a) ** 2, -1).numpy()
    m = (a[:, 0] * a[:, 0] + a[:, 1] * a[:, 1]) + a[:, 2] * a[:, 2]
    np.testing.assert_array_equal(t, m)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ball_query_numpy_matches_c_and_threshold(coracle, seed):
    import importlib
    ops = importlib.import_module("dpfm_amd.ops")
    rng = np.random.default_rng(seed)
    r = 0.05 * 13.7
    pc1, pc2 = boundary_cloud(rng, 400, 300, r)
    ref = O.find_positives(pc1, pc2, r)
    pairs, o12, o21 = c_ball_query(coracle, pc1, pc2, r)
    np.testing.assert_array_equal(ref, pairs)
    e12, e21 = O.get_overlap(400, 300, ref)
    np.testing.assert_array_equal(e12, o12)
    np.testing.assert_array_equal(e21, o21)
    # sqrt(s) <= r  <=>  s <= T(r) on the numpy sums (the kernel's test)
    d = pc1[:, None] - pc2
    s = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    np.testing.assert_array_equal(np.argwhere(s <= ops.ball_threshold(r)), ref)


def test_ball_threshold_exact():
    import importlib
    ops = importlib.import_module("dpfm_amd.ops")
    rng = np.random.default_rng(3)
    for r in list(rng.uniform(0.1, 2.0, 200)) + [0.5, 0.25, 1.0, 0.7]:
        T = ops.ball_threshold(r)
        assert math.sqrt(T) <= r
        assert math.sqrt(math.nextafter(T, math.inf)) > r


def test_erode_plus_kernel():
    m = np.zeros((6, 7), bool)
    m[1:5, 1:6] = True
    m[0, 3] = True
    e = O.erode_seg_mask(m)
    exp = np.zeros_like(m)
    exp[2:4, 2:5] = True
    exp[1, 3] = True  # plus kernel: (1,3) sees (0,3),(2,3),(1,2),(1,4) all set
    np.testing.assert_array_equal(e, exp)
    # border pixels are not eroded by the image edge (cv2 default border)
    full = np.ones((4, 4), bool)
    assert O.erode_seg_mask(full).all()


def test_transform_inverse_roundtrip():
    rng = np.random.default_rng(5)
    from dpfm_amd.dataset.synthetic import random_rotation
    R = random_rotation(rng)
    t = rng.normal(size=3) * 50
    obj = rng.normal(size=(100, 3)) * 5
    cam = O.transform(obj, R, t, inv=False)
    back = O.transform(cam, R, t, inv=True)
    np.testing.assert_allclose(back, obj, atol=1e-10)


def test_umeyama_recovers_rigid_transform(coracle):
    import ctypes
    from _util import cp
    from dpfm_amd.dataset.synthetic import random_rotation
    rng = np.random.default_rng(7)
    for _ in range(20):
        R = random_rotation(rng)
        t = rng.normal(size=3) * 30
        src = np.ascontiguousarray(rng.normal(size=(4, 3)) * 5)
        dst = np.ascontiguousarray(src @ R.T + t)
        T = O.umeyama(src.T, dst.T)
        np.testing.assert_allclose(T[:3, :3], R, atol=1e-9)
        np.testing.assert_allclose(T[:3, 3], t, atol=1e-8)
        Rc = np.zeros(9)
        tc = np.zeros(3)
        coracle.oc_umeyama(cp(src), cp(dst), 4, cp(Rc), cp(tc))
        np.testing.assert_allclose(Rc.reshape(3, 3), R, atol=1e-9)
        np.testing.assert_allclose(tc, t, atol=1e-8)


def test_ransac_c_matches_python(coracle):
    from _util import cp
    from dpfm_amd.dataset.synthetic import random_rotation
    rng = np.random.default_rng(11)
    R = random_rotation(rng)
    t = rng.normal(size=3) * 30
    src = rng.normal(size=(200, 3)) * 5
    dst = src @ R.T + t
    n = 150
    corres = np.stack([rng.integers(0, 200, n), rng.integers(0, 200, n)], 1).astype(np.int32)
    good = rng.random(n) < 0.4
    corres[good, 1] = corres[good, 0]
    dst = np.ascontiguousarray(dst + rng.normal(size=dst.shape) * 0.01)
    H = 300
    hyps = np.array([[coracle.oc_hyp_index(42, h, j, n) for j in range(4)] for h in range(H)], dtype=np.int32)
    Tp, f, rm, hb = O.ransac_registration(src, dst, corres, hyps, 0.05)
    T = np.zeros(16)
    st = np.zeros(3)
    coracle.oc_ransac(cp(np.ascontiguousarray(src)), cp(dst), cp(np.ascontiguousarray(corres)), n, None, 42, H, 0.05,
                      cp(T), cp(st))
    assert int(st[2]) == hb
    assert st[0] == f
    np.testing.assert_allclose(T.reshape(4, 4), Tp, atol=1e-9)


def test_transform_oracle_vs_numpy_literal_real_crops():
    """H4's oracle evaluates pc @ R + (-t @ R) as left-to-right 3-term dots without FMA (the
    order the HIP kernel reproduces bit-exactly). The reference's literal numpy expression
    (object.py:304-307) goes through BLAS, whose order is library-dependent. On the
    reference's real crops (tests/golden/real_crops.npz) the two differ by at most a few
    ulps of the coordinates' scale (|x| <= |pc| + |t|), and no find_positives pair flips."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "real_crops.npz"))
    flips = pairs = 0
    for k in range(int(g["n"])):
        T = g[f"{k}_T_gt"]
        R, t, pc = T[:3, :3].copy(), T[:3, 3].copy(), g[f"{k}_pc"]
        cad = g[f"cad_{int(g[f'{k}_obj_id'])}"]
        mine = O.transform(pc, R, t, inv=True)
        literal = pc @ R + (-1.0 * t.reshape(1, 3) @ R)
        scale = np.abs(pc).max() + np.abs(t).max()
        assert np.abs(mine - literal).max() <= 8 * np.finfo(np.float64).eps * scale
        r = float(g[f"{k}_diam"]) * 0.05
        a, b = O.find_positives_mask(cad, mine, r), O.find_positives_mask(cad, literal, r)
        flips += int((a != b).sum())
        pairs += int(a.sum())
    assert pairs > 200_000 and flips == 0


def _icp_case(rng, ns=300, nt=400, deg=4.0, shift=0.3):
    from dpfm_amd.dataset.synthetic import random_rotation
    tgt = rng.normal(size=(nt, 3)) * np.array([4.0, 3.0, 2.0]) + np.array([1.0, -2.0, 80.0])
    src = np.ascontiguousarray(tgt[rng.permutation(nt)[:ns]] + rng.normal(size=(ns, 3)) * 0.02)
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    a = np.deg2rad(deg)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    R = np.eye(3) + np.sin(a) * K + (1 - np.cos(a)) * K @ K
    c = src.mean(0)
    T0 = np.eye(4)
    T0[:3, :3] = R
    T0[:3, 3] = c - R @ c + rng.normal(size=3) * shift
    return src, np.ascontiguousarray(tgt), T0


@pytest.mark.parametrize("seed,max_it", [(0, 30), (1, 2000), (2, 3), (3, 0)])
def test_icp_c_matches_python(coracle, seed, max_it):
    """(f4) oc_icp (the GPU parity checker) against the numpy restatement of Open3D's ICP loop."""
    from _util import cp
    rng = np.random.default_rng(seed)
    src, tgt, T0 = _icp_case(rng)
    Tp, fp, rp, itp, cvp = O.registration_icp(src, tgt, 0.5, T0, max_it)
    T = np.zeros(16)
    st = np.zeros(4)
    coracle.oc_icp(cp(src), src.shape[0], cp(tgt), tgt.shape[0], cp(np.ascontiguousarray(T0)), 0.5, max_it, 1e-6, 1e-6,
                   cp(T), cp(st))
    assert int(st[2]) == itp and bool(st[3]) == cvp
    assert abs(st[0] - fp) < 1e-12 and abs(st[1] - rp) < 1e-9
    np.testing.assert_allclose(T.reshape(4, 4), Tp, atol=1e-9)
    if max_it >= 30:
        assert fp > 0.9 and cvp  # a 4 degree / 3 mm perturbation is recovered


def test_icp_c_no_pairs_and_empty_target(coracle):
    from _util import cp
    rng = np.random.default_rng(5)
    src, tgt, T0 = _icp_case(rng)
    T0[:3, 3] += 100.0  # far away: no pair within the radius
    for nt in (tgt.shape[0], 0):
        T = np.zeros(16)
        st = np.zeros(4)
        coracle.oc_icp(cp(src), src.shape[0], cp(tgt), nt, cp(np.ascontiguousarray(T0)), 0.5, 50, 1e-6, 1e-6,
                       cp(T), cp(st))
        np.testing.assert_array_equal(T.reshape(4, 4), T0)
        assert st[0] == 0.0 and st[1] == 0.0 and st[2] == 1 and st[3] == 1
