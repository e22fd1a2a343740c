"""Index consumers take untrusted indices without faulting (round-4 verdict: a garbage argmin
index fed to a gather aborted the process): pk_inlier_ratio, pk_gather_transform and pk_ransac
read nothing through an out-of-range index, report it per crop in their status output, and the
host wrappers turn a reported crop into PoseKernError (ops.check_index_status). In-range inputs
give status 0 and unchanged results."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_inlier_ratio_flags_out_of_range(device):
    from dpfm_amd import _lib, ops
    B, V1, V2 = 3, 200, 150
    g = torch.Generator().manual_seed(3)
    cad = torch.randn(B, V1, 3, generator=g).to(device)
    pc = torch.randn(B, V2, 3, generator=g).to(device)
    pairs = torch.stack([torch.randint(0, V1, (B, 100), generator=g), torch.randint(0, V2, (B, 100), generator=g)],
                        -1).to(device)
    pairs[:, :10, 0] = pairs[:, :10, 1]  # a few close pairs (same coordinates index range)
    npairs = torch.full((B,), 100, dtype=torch.int32, device=device)
    thr = torch.full((B,), 1.0, device=device)
    ok = ops.inlier_ratio(pairs, npairs, cad, pc, thr)  # in range: no raise
    bad = pairs.clone()
    bad[1, 5, 0] = V1 + 1000          # CAD index past the array
    bad[2, 7, 1] = -3                 # negative crop index
    bad[2, 50, 0] = 1 << 40           # far out
    with pytest.raises(_lib.PoseKernError, match=r"crop\(s\) \[1, 2\]"):
        ops.inlier_ratio(bad, npairs, cad, pc, thr)
    st = torch.full((B,), 7, dtype=torch.int32, device=device)  # caller buffer: any contents
    ir = ops.inlier_ratio(bad, npairs, cad, pc, thr, status=st)
    assert st.tolist() == [0, 1, 1]
    # the flagged pairs count as outliers, the others as before
    exp = ok.clone()
    for b, k in [(1, 5), (2, 7), (2, 50)]:
        pr = pairs[b, k]
        d = (cad[b, pr[0]] - pc[b, pr[1]]).norm()
        exp[b] -= float(d < thr[b]) / 100
    torch.testing.assert_close(ir, exp, atol=1e-6, rtol=0)
    # the point-map layout (2) as TrainStep uses it
    pm = torch.randint(0, V1, (B, V2), generator=g).to(device)
    pm[0, 3] = V1
    n2 = torch.full((B,), V2, dtype=torch.int32, device=device)
    st2 = torch.empty((B,), dtype=torch.int32, device=device)
    ops.inlier_ratio(pm, n2, cad, pc, thr, layout=2, status=st2)
    assert st2.tolist() == [1, 0, 0]


def test_gather_transform_flags_out_of_range(device):
    from dpfm_amd import _lib, ops
    F, n = 2, 300
    g = torch.Generator().manual_seed(4)
    pcd = torch.randn(F * n, 3, generator=g, dtype=torch.float64).to(device)
    off = torch.tensor([0, n, 2 * n], dtype=torch.int64, device=device)
    npoint = torch.tensor([64, 64], dtype=torch.int32, device=device)
    out_off = torch.tensor([0, 64, 128], dtype=torch.int64, device=device)
    idx = torch.randint(0, n, (F, 64), generator=g).to(device)
    R = torch.eye(3, dtype=torch.float64, device=device).reshape(1, 9).repeat(F, 1).contiguous()
    t = torch.zeros((F, 3), dtype=torch.float64, device=device)
    good = ops.gather_transform(pcd, off, idx, npoint, 64, out_off, R, t, F * 64)
    assert good["status"].tolist() == [0, 0]
    bad = idx.clone()
    bad[1, 9] = n           # one past the crop (would read crop 2's neighbour / past the array)
    with pytest.raises(_lib.PoseKernError):
        ops.gather_transform(pcd, off, bad, npoint, 64, out_off, R, t, F * 64)
    st = torch.empty((F,), dtype=torch.int32, device=device)
    r = ops.gather_transform(pcd, off, bad, npoint, 64, out_off, R, t, F * 64, status=st)
    assert st.tolist() == [0, 1]
    s64 = r["sel64"].cpu()
    assert torch.isnan(s64[64 + 9]).all() and not torch.isnan(s64[:64 + 9]).any() and not torch.isnan(s64[64 + 10:]).any()
    torch.testing.assert_close(s64[:64], good["sel64"].cpu()[:64], rtol=0, atol=0)


def test_ransac_flags_out_of_range(device):
    from dpfm_amd import _lib, ops
    rng = np.random.default_rng(5)
    B, n, H = 2, 120, 256
    cad = torch.from_numpy(rng.normal(size=(B * 80, 3))).to(device)
    pc = torch.from_numpy(rng.normal(size=(B * 60, 3))).to(device)
    src_off = torch.tensor([0, 80, 160], dtype=torch.int64, device=device)
    dst_off = torch.tensor([0, 60, 120], dtype=torch.int64, device=device)
    corres = torch.from_numpy(np.stack([rng.integers(0, 80, B * n), rng.integers(0, 60, B * n)], 1).astype(np.int32)
                              ).to(device)
    cor_off = torch.tensor([0, n, 2 * n], dtype=torch.int64, device=device)
    T0, s0 = ops.ransac(cad, src_off, pc, dst_off, corres, cor_off, H, seed=1)
    bad = corres.clone()
    bad[n + 17, 0] = 80      # crop 1: source row past its CAD
    with pytest.raises(_lib.PoseKernError, match=r"crop\(s\) \[1\]"):
        ops.ransac(cad, src_off, pc, dst_off, bad, cor_off, H, seed=1)
    st = torch.full((B,), -1, dtype=torch.int32, device=device)
    T1, s1 = ops.ransac(cad, src_off, pc, dst_off, bad, cor_off, H, seed=1, status=st)
    assert st.tolist() == [0, 1]
    torch.testing.assert_close(T1[0], T0[0], rtol=0, atol=0)  # the clean crop is unchanged
    # caller hypotheses out of range
    hy = torch.from_numpy(rng.integers(0, n, size=(B * 8, 4)).astype(np.int32)).to(device)
    hy[3, 2] = n + 5
    hoff = torch.tensor([0, 8, 16], dtype=torch.int64, device=device)
    st.fill_(9)
    ops.ransac(cad, src_off, pc, dst_off, corres, cor_off, 8, hyps=hy, hyp_off=hoff, status=st)
    assert st.tolist() == [1, 0]
