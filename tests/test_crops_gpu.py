"""GPU parity: crop formation (H1 back-projection + erosion, H2 SOR, FPS policy, H4
gather + transform) vs the oracle, on the reference's LM sample frame and on
synthetic frames. Bit-exact except where noted."""
import os

import numpy as np
import pytest
import torch

from oracle import dpfm_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _frames():
    from dpfm_amd.dataset.synthetic import make_frame
    g = np.load(os.path.join(GOLD, "lm_frame.npz"))
    depth, masks, K, ds = g["depth"], g["masks"], g["K"], float(g["depth_scale"])
    frames = []
    for j in (0, 2, 4, 7, 11, 1, 14):  # includes an empty mask (1) and a tiny one (14)
        frames.append((depth, masks[j], K, ds))
    for s in range(3):
        f = make_frame(s)
        frames.append((f.depth, f.mask, f.K, f.depth_scale))
    return frames


def test_backproject_bitexact(device):
    from dpfm_amd import ops
    fr = _frames()
    depth = torch.from_numpy(np.stack([f[0].astype(np.int16) for f in fr])).to(device)
    mask = torch.from_numpy(np.stack([f[1] for f in fr])).to(device)
    K = torch.from_numpy(np.stack([f[2].reshape(9) for f in fr])).to(device)
    cs = torch.tensor([1000.0 / f[3] for f in fr], dtype=torch.float32, device=device)
    out = ops.backproject(depth, mask, K, cs, cap=200000)
    off = out["off"].cpu().numpy()
    xyz = out["xyz"].cpu().numpy()
    for b, (d, m, k, ds) in enumerate(fr):
        exp = O.dpt_2_pcld(d, 1000 / ds, k, m == 255)
        got = xyz[off[b]:off[b + 1]]
        assert got.shape == exp.shape, b
        np.testing.assert_array_equal(got, exp, err_msg=f"frame {b}")


def _packed(arrs, device, dtype=torch.float64):
    from dpfm_amd import ops
    return (torch.from_numpy(np.concatenate(arrs, 0)).to(device=device, dtype=dtype),
            ops.packed_offsets([a.shape[0] for a in arrs], device))


def test_sor_matches_oracle(device):
    from dpfm_amd import ops
    clouds = [O.dpt_2_pcld(d, 1000 / ds, k, m == 255) for d, m, k, ds in _frames()]
    clouds = [c for c in clouds if c.shape[0] > 0]
    clouds.append(np.repeat(clouds[0][:30], 2, axis=0))  # duplicates: zero distances
    x, off = _packed(clouds, device)
    res = ops.sor(x, off, max(c.shape[0] for c in clouds), want_idx=True)
    avg = res["avg"].cpu().numpy()
    o = off.cpu().numpy()
    oo = res["off"].cpu().numpy()
    kidx = res["kept_idx"].cpu().numpy()
    x64 = res["xyz64"].cpu().numpy()
    x32 = res["xyz32"].cpu().numpy()
    for b, c in enumerate(clouds):
        exp_avg = O.sor_avg_distances(c)
        np.testing.assert_array_equal(avg[o[b]:o[b + 1]], exp_avg, err_msg=f"avg crop {b}")
        keep = O.remove_outliers_indices(c)
        np.testing.assert_array_equal(kidx[oo[b]:oo[b + 1]], keep, err_msg=f"keep crop {b}")
        np.testing.assert_array_equal(x64[oo[b]:oo[b + 1]], c[keep])
        np.testing.assert_array_equal(x32[oo[b]:oo[b + 1]], c[keep].astype(np.float32))


@pytest.mark.parametrize("fixed", [0, 1024])
def test_npoint_fps_gather_transform(device, coracle, fixed):
    from dpfm_amd import ops
    from dpfm_amd.dataset.synthetic import make_frame, random_rotation
    from _util import c_fps
    rng = np.random.default_rng(4)
    clouds = []
    for s in range(4):
        f = make_frame(s)
        c = O.dpt_2_pcld(f.depth, 1000 / f.depth_scale, f.K, f.mask == 255)
        clouds.append(c)
    clouds.append(clouds[0][:1500])  # n <= 2000: no FPS in reference mode
    x, off = _packed(clouds, device)
    pol = ops.fps_npoint(off, fixed=fixed, limit=2000, seed=7)
    npoint = pol["npoint"].cpu().numpy()
    start = pol["start"].cpu().numpy()
    for b, c in enumerate(clouds):
        n = c.shape[0]
        if fixed:
            assert npoint[b] == fixed
        elif n > 2000:
            assert npoint[b] == O.fps_npoint(n)
        else:
            assert npoint[b] == -n
    x32 = x.to(torch.float32)
    npmax = int(np.abs(npoint).max())
    idx = ops.fps_packed(x32, off, max(c.shape[0] for c in clouds), pol["start"], pol["npoint"], npmax)
    R = np.stack([random_rotation(rng) for _ in clouds])
    t = rng.normal(size=(len(clouds), 3)) * 40
    total = int(np.abs(npoint).sum())
    g = ops.gather_transform(x, off, idx, pol["npoint"], npmax, pol["off"],
                             torch.from_numpy(R.reshape(-1, 9)).to(device), torch.from_numpy(t).to(device), total)
    oo = pol["off"].cpu().numpy()
    idx = idx.cpu().numpy()
    for b, c in enumerate(clouds):
        if npoint[b] > 0:
            exp_idx = c_fps(coracle, c.astype(np.float32), start[b], npoint[b])
            np.testing.assert_array_equal(idx[b, :npoint[b]], exp_idx)
            sel = c[exp_idx]
        else:
            sel = c
        np.testing.assert_array_equal(g["sel64"].cpu().numpy()[oo[b]:oo[b + 1]], sel)
        np.testing.assert_array_equal(g["sel32"].cpu().numpy()[oo[b]:oo[b + 1]], sel.astype(np.float32))
        np.testing.assert_array_equal(g["align"].cpu().numpy()[oo[b]:oo[b + 1]], O.transform(sel, R[b], t[b], inv=True))


@pytest.mark.parametrize("with_K", [False, True])
def test_sor_pixel_window_path_bitexact(device, with_K):
    """backproject -> sor with the pixel-window kNN bound (and, with K, the camera-model
    pixel box) gives the brute-force result."""
    from dpfm_amd import ops
    fr = _frames()
    depth = torch.from_numpy(np.stack([f[0].astype(np.int16) for f in fr])).to(device)
    mask = torch.from_numpy(np.stack([f[1] for f in fr])).to(device)
    K = torch.from_numpy(np.stack([f[2].reshape(9) for f in fr])).to(device)
    cs = torch.tensor([1000.0 / f[3] for f in fr], dtype=torch.float32, device=device)
    bp = ops.backproject(depth, mask, K, cs, cap=200000)
    nmax = int((bp["off"][1:] - bp["off"][:-1]).max())
    res = ops.sor(bp["xyz"], bp["off"], nmax, pix=bp["pix"], idxmap=bp["idxmap"], want_idx=True,
                  K=K if with_K else None)
    off = bp["off"].cpu().numpy()
    oo = res["off"].cpu().numpy()
    avg = res["avg"].cpu().numpy()
    kidx = res["kept_idx"].cpu().numpy()
    xyz = bp["xyz"].cpu().numpy()
    for b in range(len(fr)):
        c = xyz[off[b]:off[b + 1]]
        if c.shape[0] == 0:
            continue
        np.testing.assert_array_equal(avg[off[b]:off[b + 1]], O.sor_avg_distances(c), err_msg=f"frame {b}")
        np.testing.assert_array_equal(kidx[oo[b]:oo[b + 1]], O.remove_outliers_indices(c))


def _seq_sum(v):
    s = 0.0
    for x in v.tolist():
        s = s + x  # IEEE double, round to nearest even, in order
    return s


def test_sor_ordered_sum_exact(device):
    """The SOR statistics' ordered fp64 sums (std::accumulate order, object.py:33-50 via
    Open3D) computed by binade-wise integer scans (crop.hip seq_sum_exact) equal the
    sequential sum bit for bit: random magnitudes, zeros, exact ties (terms of half an ulp
    of the running sum), terms larger than the sum, and every binade crossing."""
    from dpfm_amd import _lib
    rng = np.random.default_rng(11)
    cases = [np.zeros(0), np.array([3.0]), rng.random(5), rng.random(256), rng.random(257),
             rng.random(1000) * 7.3, rng.random(20000) * 0.01 + 1.0, rng.exponential(size=100000),
             np.concatenate([np.zeros(3000), rng.random(9000)]),
             np.concatenate([[2.0 ** 52], np.full(3000, 0.5), [1.5, 2.5, 0.5, 3.5]]),
             np.concatenate([[2.0 ** 40], rng.integers(0, 8, 12000) * 2.0 ** -13]),
             np.concatenate([rng.random(300), [1e300], rng.random(9000), [1e-300] * 50]),
             np.ldexp(rng.integers(1, 2 ** 20, 30000).astype(np.float64), rng.integers(-30, 5, 30000)),
             rng.random(12000) ** 8]
    for i, v in enumerate(cases):
        v = np.ascontiguousarray(v, dtype=np.float64)
        t = torch.from_numpy(v).to(device)
        out = torch.empty(1, dtype=torch.float64, device=device)
        assert _lib.dev_lib().pkdev_seq_sum(_lib.ptr(t), int(v.size), _lib.ptr(out), _lib.stream(device)) == 0
        got = float(out.cpu()[0])
        exp = _seq_sum(v)
        assert got == exp, (i, got, exp, got - exp)


def test_sor_threshold_bitexact(device):
    """sor's per-crop threshold mean + 0.3 std equals the ordered-sum restatement exactly."""
    from dpfm_amd import ops
    import math
    clouds = [O.dpt_2_pcld(d, 1000 / ds, k, m == 255) for d, m, k, ds in _frames()]
    clouds = [c for c in clouds if c.shape[0] > 0]
    x, off = _packed(clouds, device)
    res = ops.sor(x, off, max(c.shape[0] for c in clouds), want_idx=True)
    assert "thr" in res
    thr = res["thr"].cpu().numpy()
    for b, c in enumerate(clouds):
        avg = O.sor_avg_distances(c)
        n = avg.size
        s = _seq_sum(np.where(avg > 0, avg, 0.0))
        mean = s / n
        ss = _seq_sum(np.where(avg > 0, (avg - mean) * (avg - mean), 0.0))
        exp = mean + 0.3 * math.sqrt(ss / (n - 1))
        assert thr[b] == exp, (b, thr[b], exp)


@pytest.mark.gpu
@pytest.mark.parametrize("fixed", [0, 1024])
def test_fps_npoint_many_crops(device, fixed):
    """pk_fps_npoint over 150 crops (three 64-crop chunks of the one-wave kernel): the policy per
    crop, the start draw splitmix64(seed ^ splitmix64(base + b)) % n, and the packed offsets as
    the running sum of |npoint| (the chunk carry)."""
    from dpfm_amd import ops
    rng = np.random.default_rng(5)
    counts = rng.integers(0, 6000, 150)
    counts[[3, 70, 140]] = 0
    off = torch.from_numpy(np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)).to(device)
    seed, base = 11, 1000
    pol = ops.fps_npoint(off, fixed=fixed, limit=2000, seed=seed, base=base)
    npoint = pol["npoint"].cpu().numpy()
    start = pol["start"].cpu().numpy()
    oo = pol["off"].cpu().numpy()
    M = (1 << 64) - 1

    def sm(x):
        x = (x + 0x9E3779B97F4A7C15) & M
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
        return x ^ (x >> 31)
    acc = 0
    for b, n in enumerate(counts.tolist()):
        if fixed:
            exp = fixed if n > fixed else -n
        else:
            exp = O.fps_npoint(n) if n > 2000 else -n
        assert npoint[b] == exp, b
        assert start[b] == (sm(seed ^ sm(base + b)) % n if n > 0 else 0), b
        assert oo[b] == acc, b
        acc += abs(exp)
    assert oo[150] == acc


@pytest.mark.gpu
@pytest.mark.parametrize("W", [633, 1100])
def test_backproject_odd_widths_and_index_map(device, W):
    """pk_backproject at row widths off the 16-pixel vector path (633) and past one 1024-pixel
    segment (1100): points bit-exact vs the oracle, and pix / idxmap consistent with them."""
    from dpfm_amd import ops
    fr = _frames()
    rng = np.random.default_rng(W)
    ds, ms = [], []
    for d, m, k, s_ in fr[:4] + fr[-2:]:
        dd = np.zeros((d.shape[0], W), d.dtype)
        mm = np.zeros((m.shape[0], W), m.dtype)
        c = min(W, d.shape[1])
        dd[:, :c], mm[:, :c] = d[:, :c], m[:, :c]
        if W > d.shape[1]:  # the extra columns: a mirrored copy of the frame's right part
            e = W - d.shape[1]
            dd[:, c:], mm[:, c:] = d[:, -e:][:, ::-1], m[:, -e:][:, ::-1]
        mm[rng.random(mm.shape) < 0.002] = 0  # holes: erosion at scattered pixels
        ds.append(dd)
        ms.append(mm)
    sel = fr[:4] + fr[-2:]
    depth = torch.from_numpy(np.stack([x.astype(np.int16) for x in ds])).to(device)
    mask = torch.from_numpy(np.stack(ms)).to(device)
    K = torch.from_numpy(np.stack([f[2].reshape(9) for f in sel])).to(device)
    cs = torch.tensor([1000.0 / f[3] for f in sel], dtype=torch.float32, device=device)
    out = ops.backproject(depth, mask, K, cs, cap=400000)
    off = out["off"].cpu().numpy()
    xyz = out["xyz"].cpu().numpy()
    pix = out["pix"].cpu().numpy()
    idxmap = out["idxmap"].cpu().numpy()
    H = ds[0].shape[0]
    for b in range(len(sel)):
        exp = O.dpt_2_pcld(ds[b], 1000 / sel[b][3], sel[b][2], ms[b] == 255)
        got = xyz[off[b]:off[b + 1]]
        assert got.shape == exp.shape, b
        np.testing.assert_array_equal(got, exp, err_msg=f"frame {b}")
        p = pix[off[b]:off[b + 1]]
        im = idxmap[b].reshape(H, W)
        assert (im.reshape(-1)[p] == np.arange(p.shape[0])).all(), b
        assert (im >= 0).sum() == p.shape[0], b


@pytest.mark.gpu
def test_gather_transform_pad_equals_gather_then_collate(device):
    """pk_gather_transform_pad's padded f32 fields and counts are exactly pk_collate_pad of the
    packed gather outputs (ld above and below the largest crop), and its packed outputs equal
    pk_gather_transform's."""
    from dpfm_amd import ops
    from dpfm_amd.dataset.synthetic import random_rotation
    rng = np.random.default_rng(9)
    counts = [700, 0, 1500, 1024, 33]
    clouds = [rng.normal(size=(n, 3)) * 20 + 100 for n in counts]
    x, off = _packed(clouds, device)
    pol = ops.fps_npoint(off, fixed=1024, limit=2000, seed=3)
    npmax = 1024
    idx = ops.fps_packed(x.to(torch.float32), off, max(counts), pol["start"], pol["npoint"], npmax)
    R = torch.from_numpy(np.stack([random_rotation(rng) for _ in counts]).reshape(-1, 9)).to(device)
    t = torch.from_numpy(rng.normal(size=(len(counts), 3)) * 40).to(device)
    total = int(pol["npoint"].abs().sum())
    st = torch.empty((len(counts),), dtype=torch.int32, device=device)
    a = ops.gather_transform(x, off, idx, pol["npoint"], npmax, pol["off"], R, t, total, want_sel32=False, status=st)
    for ld in (1024, 600, 1100):
        st2 = torch.empty_like(st)
        b = ops.gather_transform(x, off, idx, pol["npoint"], npmax, pol["off"], R, t, total, want_sel32=False,
                                 status=st2, pad_ld=ld)
        assert torch.equal(a["sel64"], b["sel64"]) and torch.equal(a["align"], b["align"])
        pc, n2 = ops.collate_pad(a["sel64"], pol["off"], ld)
        al, _ = ops.collate_pad(a["align"], pol["off"], ld)
        assert torch.equal(b["pc32"], pc) and torch.equal(b["align32"], al) and torch.equal(b["n2"], n2), ld
