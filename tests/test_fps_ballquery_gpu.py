"""GPU parity: FPS (H3) and ball query (H5) kernels vs the oracle, bit-exact."""
import numpy as np
import pytest
import torch

from oracle import dpfm_oracle as O
from _util import c_fps, boundary_cloud

pytestmark = pytest.mark.gpu


def _packed(arrs, dtype, device):
    from dpfm_amd import ops
    flat = np.concatenate(arrs, 0).astype(dtype)
    return torch.from_numpy(flat).to(device), ops.packed_offsets([a.shape[0] for a in arrs], device)


@pytest.mark.parametrize("sizes,grid", [
    ([1, 7, 100, 1024, 2049, 4500, 9000, 13000, 14000, 20000, 26000], False),  # > 13312: per-lane buckets, plain
    ([1, 7, 100, 1024, 2049, 4500, 9000, 13000], False),         # pruned buckets, random order
    ([500, 3000, 8000, 13312], True),                             # pruned, spatially coherent runs
    ([300, 2649, 5100, 9289], True),                              # 10 points per lane (<= 10,240)
    ([9, 600, 10240], False),
])
def test_fps_ragged_batch_bitexact(device, coracle, sizes, grid):
    from dpfm_amd import ops
    rng = np.random.default_rng(0)
    crops = []
    for n in sizes:
        if grid:  # row-major samples of a bumpy surface, like back-projected pixels
            w = int(np.ceil(np.sqrt(n)))
            v, u = np.divmod(np.arange(n), w)
            z = 100 + 3 * np.sin(u / 9.0) * np.cos(v / 7.0)
            x = np.stack([(u - w / 2) * 0.15, (v - w / 2) * 0.15, z], 1).astype(np.float32)
        else:
            x = (rng.normal(size=(n, 3)) * 6 + np.array([1.0, -2.0, 110.0])).astype(np.float32)
        if n > 50:  # duplicates -> ties resolved to the lowest index
            x[rng.integers(0, n, n // 10)] = x[rng.integers(0, n, n // 10)]
        crops.append(x)
    xyz, off = _packed(crops, np.float32, device)
    start = np.array([int(rng.integers(0, n)) for n in sizes], dtype=np.int32)
    npoint = np.array([min(n, 1024) if n < 2000 else O.fps_npoint(n) for n in sizes], dtype=np.int32)
    npoint[1] = 12  # more samples than points: distances all reach 0 -> index 0 repeats
    out = ops.fps_packed(xyz, off, max(sizes), torch.from_numpy(start).to(device),
                         torch.from_numpy(npoint).to(device), int(npoint.max())).cpu().numpy()
    for b, x in enumerate(crops):
        exp = c_fps(coracle, x, start[b], npoint[b])
        np.testing.assert_array_equal(out[b, :npoint[b]], exp, err_msg=f"crop {b} (n={sizes[b]})")
        assert (out[b, npoint[b]:] == 0).all(), f"crop {b}: the row's tail is written as zeros"


def test_fps_reference_signature(device):
    from dpfm_amd.dpfm_utils import farthest_point_sample
    rng = np.random.default_rng(1)
    pcd = rng.normal(size=(2345, 3)) * 5 + 100  # f64 like the dataset's pcd
    xyz32 = torch.Tensor(pcd).t()               # dataset/object.py:147
    ratio = 2000 / pcd.shape[0]
    got = farthest_point_sample(xyz32.to(device), ratio=ratio, start=17).cpu()
    exp = O.farthest_point_sample(xyz32, ratio=ratio, start=17)
    assert got.shape[0] == O.fps_npoint(2345)
    assert torch.equal(got, exp)


@pytest.mark.parametrize("with_mask", [True, False])
def test_ball_query_bitexact(device, with_mask):
    from dpfm_amd import ops
    rng = np.random.default_rng(2)
    sizes = [(1024, 1024), (37, 999), (2048, 1500), (5002, 1999), (0, 10), (10, 0), (3, 3)]
    cads, pcs, rs = [], [], []
    for b, (n1, n2) in enumerate(sizes):
        r = 0.05 * rng.uniform(8, 20)
        if n1 and n2:
            c, p = boundary_cloud(rng, n1, n2, r)
        else:
            c, p = rng.normal(size=(n1, 3)), rng.normal(size=(n2, 3))
        cads.append(c)
        pcs.append(p)
        rs.append(r)
    cad, coff = _packed(cads, np.float64, device)
    pc, poff = _packed(pcs, np.float64, device)
    n1max = max(s[0] for s in sizes)
    n2max = max(s[1] for s in sizes)
    cap = 200000
    res = ops.ball_query(cad, coff, pc, poff, rs, n1max, n2max, cap, with_mask=with_mask)
    ops.check_capacity(res["count"], cap)
    assert int(res["overflow"]) == 0  # the kernel's flag: no crop above cap
    count = res["count"].cpu().numpy()
    pairs = res["pairs"].cpu().numpy()
    o12 = res["overlap_12"].cpu().numpy()
    o21 = res["overlap_21"].cpu().numpy()
    mask = res["mask"].cpu().numpy() if with_mask else None
    for b, (c, p, r) in enumerate(zip(cads, pcs, rs)):
        n1, n2 = c.shape[0], p.shape[0]
        if n1 and n2:
            exp = O.find_positives(c, p, r)
        else:
            exp = np.zeros((0, 2), dtype=np.int64)
        assert count[b] == exp.shape[0], f"crop {b}"
        np.testing.assert_array_equal(pairs[b, :count[b]], exp, err_msg=f"crop {b}")
        e12, e21 = O.get_overlap(n1, n2, exp) if exp.size else (np.zeros(n1, np.int8), np.zeros(n2, np.int8))
        np.testing.assert_array_equal(o12[b, :n1], e12)
        np.testing.assert_array_equal(o21[b, :n2], e21)
        if mask is not None and n1 and n2:
            np.testing.assert_array_equal(mask[b, :n1, :n2].astype(bool), O.find_positives_mask(c, p, r))
            assert not mask[b, :n1, n2:].any()


def test_ball_query_capacity_overflow_reported(device):
    from dpfm_amd import ops, _lib
    rng = np.random.default_rng(3)
    c = rng.normal(size=(64, 3)) * 0.01
    p = rng.normal(size=(64, 3)) * 0.01
    cad, coff = _packed([c], np.float64, device)
    pc, poff = _packed([p], np.float64, device)
    res = ops.ball_query(cad, coff, pc, poff, [1.0], 64, 64, 100)
    assert int(res["count"][0]) == 64 * 64
    assert int(res["overflow"]) == 1  # pk_ball_query_pairs' device flag (Crops.overflow)
    with pytest.raises(_lib.PoseKernError):
        ops.check_capacity(res["count"], 100)
    exp = O.find_positives(c, p, 1.0)[:100]
    np.testing.assert_array_equal(res["pairs"][0].cpu().numpy(), exp)


@pytest.mark.parametrize("cap", [100, 1 << 16])
def test_ball_query_colcount_and_cgt_from_it(device, cap):
    """pk_ball_query_pairs' colcount (pairs per crop point among the kept list, integer atomics)
    equals a bincount of the kept pairs' crop indices, truncated lists included; pk_cgt_lstsq fed
    with it returns bit for bit what it returns counting the pairs itself (same fp64 sums)."""
    from dpfm_amd import ops
    rng = np.random.default_rng(11)
    cs = [rng.normal(size=(n, 3)) * 2 for n in (300, 64, 1)]
    ps = [rng.normal(size=(n, 3)) * 2 for n in (250, 64, 5)]
    cad, coff = _packed(cs, np.float64, device)
    pc, poff = _packed(ps, np.float64, device)
    n1max, n2max = 300, 250
    res = ops.ball_query(cad, coff, pc, poff, [1.0, 3.0, 0.5], n1max, n2max, cap)
    cc = res["colcount"].cpu().numpy()
    for b in range(3):
        k = min(int(res["count"][b]), cap)
        exp = np.bincount(res["pairs"][b, :k, 1].cpu().numpy(), minlength=n2max)
        np.testing.assert_array_equal(cc[b], exp)
    g = torch.Generator().manual_seed(3)
    e1 = torch.randn(3, n1max, 32, generator=g).to(device)
    e2 = torch.randn(3, n2max, 32, generator=g).to(device)
    a = ops.cgt_lstsq(res["pairs"], res["count"], e1, e2)
    b_ = ops.cgt_lstsq(res["pairs"], res["count"], e1, e2, cnt=res["colcount"])
    assert torch.equal(a, b_)
