"""GPU parity at the BASELINE configs' own sizes (BASELINE.json configs[1], [3], [4]):

  configs[1]  B = 32 x 1024-point inference: InferStep (eval.py:73-89 + test_RANSAC.py:
              397-401) checked stage by stage against the per-crop oracle chain — model
              output C, top-5 candidates, rigidity survivors (n = 5120 per crop), IR, RANSAC
              (1024 hypotheses, same draws) and the pose metrics
  configs[3]  the feature distance at 2048^2 (B = 8 crops here) and the rigidity filter at
              n = 10240 (5 x 2048 candidates)
  configs[4]  the 4096^2 feature distance (one crop) and 1024-hypothesis RANSAC over
              n = 4096 correspondences
Index outputs are exact except counted near-ties, the rule of SURVEY §8(c)."""
import numpy as np
import pytest
import torch

from oracle import dpfm_oracle as O
from oracle import dpfm_model_oracle as M
from _util import check_topk, rigidity_parity as _rigidity_parity, train_step_parity

pytestmark = pytest.mark.gpu


def _spectral(V, seed):
    from dpfm_amd.dataset.synthetic import lbo_operators
    return torch.from_numpy(lbo_operators(V, 64, seed)[2])


@pytest.mark.parametrize("B,V", [(8, 2048), (1, 4096)])
def test_feat_dist_argmin_top5_configs(device, B, V):
    """naive.py:20-33 (argmin) and spacial_filtering.py:19-38 (top-5 of the stable sort) on
    the MFMA kernel vs torch.cdist on the CPU, at configs[3]'s 2048^2 and configs[4]'s 4096^2."""
    from dpfm_amd import ops
    torch.manual_seed(B)
    ex = torch.stack([_spectral(V, 100 + b) for b in range(B)])
    ey = torch.stack([_spectral(V, 200 + b) for b in range(B)])
    C = torch.eye(30)[None] + 0.3 * torch.randn(B, 30, 30)
    n = torch.full((B,), V, dtype=torch.int32, device=device)
    i1, _ = ops.feat_dist_topk(ex.to(device), C.to(device), ey.to(device), n, n, 1)
    i5, d5 = ops.feat_dist_topk(ex.to(device), C.to(device), ey.to(device), n, n, 5, want_dist=True)
    i1, i5, d5 = i1.cpu().numpy(), i5.cpu().numpy(), d5.cpu().numpy()
    ties = 0
    for b in range(B):
        dist = torch.cdist(ex[b, :, :30] @ C[b].t(), ey[b, :, :30]).numpy().astype(np.float64)
        ties += check_topk(dist, i1[b], 1) + check_topk(dist, i5[b], 5)
        picked = np.take_along_axis(dist, i5[b].T, axis=0).T
        np.testing.assert_allclose(d5[b], picked, rtol=1e-4, atol=1e-5 * dist.max())
    assert ties <= max(2, B * V // 1000), ties


def test_feat_dist_scratch_contents_do_not_matter(device):
    """pk_feat_dist_topk keeps nothing in its scratch across calls (posekern.h): every call of a
    sequence of layouts (top-1 fp32 with and without row parts, bf16 / bf16x3, top-5) gives the
    same result on a zeroed buffer, on one filled with 0xFF and on one of random bytes, each call
    interleaved with the others on the same garbage buffers (the round-4 abort: stale arrival
    words from another layout left a column group unmerged)."""
    from dpfm_amd import _lib, ops
    g = torch.Generator().manual_seed(77)

    def inputs(B, V):
        ex = torch.randn(B, V, 32, generator=g).to(device)
        ey = torch.randn(B, V, 32, generator=g).to(device)
        C = torch.randn(B, 30, 30, generator=g).to(device)
        n = torch.full((B,), V, dtype=torch.int32, device=device)
        return ex, C, ey, n

    seq = [(2, 300, 1, "fp32"), (4, 512, 1, "bf16"), (32, 1024, 1, "fp32"), (3, 700, 5, "fp32"),
           (8, 2048, 1, "fp32"), (1, 4096, 1, "fp32"), (4, 4096, 1, "bf16x3"), (32, 1024, 1, "fp32")]
    cases = [(inputs(B, V), B, V, k, prec) for B, V, k, prec in seq]
    nmax = max(int(_lib.lib().pk_feat_dist_work_size(B, V, V, k, ops.FD_MODES[p])) for _, B, V, k, p in cases)
    ff = torch.full((nmax + 4096,), 0xFF, dtype=torch.uint8, device=device)
    rnd = torch.randint(0, 256, (nmax + 4096,), dtype=torch.uint8, generator=g).to(device)
    refs = []
    for (ex, C, ey, n), B, V, k, prec in cases:
        nb = int(_lib.lib().pk_feat_dist_work_size(B, V, V, k, ops.FD_MODES[prec]))
        ref, _ = ops.feat_dist_topk(ex, C, ey, n, n, k, precision=prec,
                                    work=torch.zeros(max(nb, 1), dtype=torch.uint8, device=device))
        refs.append(ref)
    for rep in range(2):
        for ((ex, C, ey, n), B, V, k, prec), ref in zip(cases, refs):
            for buf in (ff, rnd):
                got, _ = ops.feat_dist_topk(ex, C, ey, n, n, k, precision=prec, work=buf)
                assert torch.equal(got, ref), (B, V, k, prec, rep)
            got, _ = ops.feat_dist_topk(ex, C, ey, n, n, k, precision=prec)  # default temporary
            assert torch.equal(got, ref), (B, V, k, prec, rep)
    assert (refs[0] >= 0).all() and (refs[0] < 300).all()


def test_feat_dist_clamp_and_duplicate_rows(device):
    """torch.cdist's clamp_min(1e-30) tie rule on the one-launch argmin: with C = I and crop
    features equal to CAD rows, the matching distances are rounding noise around 0 (some at or
    below the clamp, which the kernel resolves by its rescan), and every such CAD row is
    duplicated at a later row: the argmin must be the first copy, clamped or not. Batches with
    and without row parts (RS > 1)."""
    from dpfm_amd import ops
    for B, V in [(32, 512), (2, 600)]:
        g = torch.Generator().manual_seed(B)
        ex = torch.randn(B, V, 32, generator=g)
        ey = torch.randn(B, V, 32, generator=g)
        C = torch.eye(30).repeat(B, 1, 1)
        expect = {}
        for b in range(B):
            src = torch.randperm(V // 2, generator=g)[:40]
            dup = V // 2 + torch.randperm(V // 2, generator=g)[:40]
            cols = torch.randperm(V, generator=g)[:40]
            ex[b, dup] = ex[b, src]
            ey[b, cols] = ex[b, src]
            for j, i in zip(cols.tolist(), src.tolist()):
                expect[(b, j)] = i
        n = torch.full((B,), V, dtype=torch.int32, device=device)
        idx, dist = ops.feat_dist_topk(ex.to(device), C.to(device), ey.to(device), n, n, 1, want_dist=True)
        idx, dist = idx[..., 0].cpu(), dist[..., 0].cpu()
        clamped = 0
        for (b, j), i in expect.items():
            assert idx[b, j].item() == i, (B, V, b, j, idx[b, j].item(), i)
            clamped += int(abs(dist[b, j].item() - 1e-15) < 1e-18)
        assert clamped > 0  # the rescan ran
        # the other columns still match cdist (near-ties counted)
        i1 = idx.numpy()
        ties = 0
        for b in range(B):
            d = torch.cdist(ex[b, :, :30], ey[b, :, :30]).numpy().astype(np.float64)
            keep = np.array([(b, j) not in expect for j in range(V)])
            ties += check_topk(d[:, keep], i1[b, keep][:, None], 1)
        assert ties <= 4, ties


def test_feat_dist_ragged_edges(device):
    """The feature-distance passes on a ragged batch whose per-crop sizes straddle the 16-row
    tile, the 4-tile register chunk and the two row halves of a block (n1, n2 in 1 .. 301):
    argmin / top-5 vs cdist on each crop's valid block (near-ties counted as above); with fewer
    than 5 valid rows the top-5 list holds them in order, then -1."""
    from dpfm_amd import ops
    sizes = [(1, 1), (1, 301), (301, 1), (15, 16), (16, 17), (17, 15), (64, 65), (65, 129), (129, 64),
             (200, 200), (5, 300), (300, 5)]
    B, V1, V2 = len(sizes), 320, 320
    g = torch.Generator().manual_seed(11)
    ex = torch.stack([_spectral(V1, 300 + b) for b in range(B)])
    ey = torch.stack([_spectral(V2, 400 + b) for b in range(B)])
    C = torch.eye(30)[None] + 0.3 * torch.randn(B, 30, 30, generator=g)
    n1 = torch.tensor([a for a, _ in sizes], dtype=torch.int32, device=device)
    n2 = torch.tensor([c for _, c in sizes], dtype=torch.int32, device=device)
    i1, _ = ops.feat_dist_topk(ex.to(device), C.to(device), ey.to(device), n1, n2, 1)
    i5, _ = ops.feat_dist_topk(ex.to(device), C.to(device), ey.to(device), n1, n2, 5)
    i1, i5 = i1.cpu().numpy(), i5.cpu().numpy()
    ties = 0
    for b, (a, c) in enumerate(sizes):
        dist = torch.cdist(ex[b, :a, :30] @ C[b].t(), ey[b, :c, :30]).numpy().astype(np.float64)
        ties += check_topk(dist, i1[b, :c], 1)
        if a >= 5:
            ties += check_topk(dist, i5[b, :c], 5)
        else:  # fewer than 5 rows: the valid ones in order, then -1
            assert (i5[b, :c, a:] == -1).all()
            srt = np.argsort(dist, axis=0, kind="stable")[:a].T
            picked = np.take_along_axis(dist, i5[b, :c, :a].T, axis=0)
            assert np.allclose(picked, np.take_along_axis(dist, srt.T, axis=0), rtol=1e-5, atol=1e-6)
    assert ties <= 3, ties


def _rigid_scene(V2, seed):
    from dpfm_amd.dataset.synthetic import random_rotation
    rng = np.random.default_rng(seed)
    V1 = V2 + 300
    cad = (rng.normal(size=(V1, 3)) * 5).astype(np.float32)
    gen = rng.permutation(V1)[:V2]
    R = random_rotation(rng)
    pc = ((cad[gen].astype(np.float64) @ R.T + np.array([3.0, -2.0, 90.0])) + rng.normal(size=(V2, 3)) * 0.05
          ).astype(np.float32)
    cand = np.zeros((V2, 5, 2), dtype=np.int64)
    cand[:, :, 1] = np.arange(V2)[:, None]
    cand[:, :, 0] = rng.integers(0, V1, size=(V2, 5))
    good = rng.random(V2) < 0.6
    cand[good, rng.integers(0, 5, size=good.sum()), 0] = gen[good]
    return cad, pc, cand.reshape(-1, 2), 2.0 * 5 * 2.5


@pytest.mark.parametrize("V2", [1024, 2048])
def test_rigidity_filter_configs(device, V2):
    """spacial_filtering.py:42-75 at n = 5 V2 = 5120 (configs[1]) and 10240 (configs[3])."""
    from dpfm_amd import ops
    cad, pc, cand, diam = _rigid_scene(V2, V2)
    thr = ops.rigidity_thresholds([diam], device)
    rows, n = ops.rigidity_filter(torch.from_numpy(cand)[None].to(device),
                                  torch.tensor([cand.shape[0]], dtype=torch.int32, device=device),
                                  torch.from_numpy(cad)[None].to(device), torch.from_numpy(pc)[None].to(device), thr)
    kept = _rigidity_parity(cad, pc, cand, rows[0].cpu().numpy(), int(n[0]), diam)
    assert 0.2 * V2 < kept < 5 * V2


def test_rigidity_filter_ragged_batch(device):
    """Crops with different candidate counts in one launch (empty, single, tile-edge ±1 of the
    256-entry pair tiles and of the first round's 320-entry group tiles, partial last groups,
    and multi-tile crops): each crop's survivors vs the oracle."""
    from dpfm_amd import ops
    sizes = [0, 1, 127, 255, 257, 319, 321, 642, 1000]
    scenes = [_rigid_scene(max((s + 4) // 5, 1), 7 + i) for i, s in enumerate(sizes)]
    Lc = max(sizes)
    cand = np.zeros((len(sizes), Lc, 2), dtype=np.int64)
    cads, pcs = [], []
    for i, (s, sc) in enumerate(zip(sizes, scenes)):
        cand[i, :s] = sc[2][:s]
        cads.append(np.pad(sc[0], ((0, 600 - sc[0].shape[0]), (0, 0))))
        pcs.append(np.pad(sc[1], ((0, 600 - sc[1].shape[0]), (0, 0))))
    dcand = torch.from_numpy(cand).to(device)
    ncand = torch.tensor(sizes, dtype=torch.int32, device=device)
    dcad = torch.from_numpy(np.stack(cads)).to(device)
    dpc = torch.from_numpy(np.stack(pcs)).to(device)
    thr = ops.rigidity_thresholds([sc[3] for sc in scenes], device)
    rows, n = ops.rigidity_filter(dcand, ncand, dcad, dpc, thr)
    rows, n = rows.cpu().numpy(), n.cpu().numpy()
    assert n[0] == 0
    for i, (s, sc) in enumerate(zip(sizes, scenes)):
        if s == 0:
            continue
        _rigidity_parity(sc[0], sc[1], sc[2][:s], rows[i], int(n[i]), sc[3])


def _rigid_dev(dl, variant, cand, ncand, cad, pc, thr):
    """pk_rigidity_filter of the dev library under pkdev_rigidity_variant(variant): (survivor
    rows, counts, the last round's scores)."""
    from dpfm_amd import _lib
    B, L, _ = cand.shape
    dev = cand.device
    la, lb = (torch.zeros((B, L), dtype=torch.int64, device=dev) for _ in range(2))
    na, nb = (torch.empty((B,), dtype=torch.int32, device=dev) for _ in range(2))
    score = torch.zeros((B, L), dtype=torch.float32, device=dev)
    part = torch.empty((max(int(dl.pk_rigidity_filter_work_size(B, L, L)) // 4, 1),), dtype=torch.float32,
                       device=dev)
    old = dl.pkdev_rigidity_variant(variant)
    try:
        rc = dl.pk_rigidity_filter(_lib.ptr(cand), L, _lib.ptr(ncand), _lib.ptr(cad), cad.shape[1], _lib.ptr(pc),
                                   pc.shape[1], _lib.ptr(thr), B, L, _lib.ptr(la), _lib.ptr(lb), _lib.ptr(na),
                                   _lib.ptr(nb), _lib.ptr(score), _lib.ptr(part), _lib.stream(dev))
        torch.cuda.synchronize()
    finally:
        dl.pkdev_rigidity_variant(old)
    assert rc == 0
    return lb.cpu(), nb.cpu(), score.cpu()


@pytest.mark.parametrize("case", ["configs3", "ragged", "split_group"])
def test_rigidity_run_tables_bit_identical(device, case):
    """Rounds 2 / 3 look the crop distance up in a run-pair table when a tile pair's crop-point
    runs are few (rigid_pair2_kernel): the pair values, scores and survivors must be the same bits
    as with both distances per pair (pkdev_rigidity_variant 3), on the configs[3] size, a ragged
    batch and a list with a split group."""
    import ctypes
    from dpfm_amd import _lib, ops
    dl = _lib.dev_lib()
    dl.pkdev_rigidity_variant.argtypes = [ctypes.c_int]
    if case == "configs3":
        scenes = [_rigid_scene(2048, 300 + b) for b in range(2)]
        sizes = [s[2].shape[0] for s in scenes]
    else:
        sizes = [1, 257, 642, 1000, 1500] if case == "ragged" else [2000]
        scenes = [_rigid_scene(max((s + 4) // 5, 1), 40 + i) for i, s in enumerate(sizes)]
    Lc, V1 = max(sizes), max(sc[0].shape[0] for sc in scenes)
    V2 = max(sc[1].shape[0] for sc in scenes)
    cand = np.zeros((len(sizes), Lc, 2), dtype=np.int64)
    for i, (s, sc) in enumerate(zip(sizes, scenes)):
        cand[i, :s] = sc[2][:s]
    if case == "split_group":
        cand[0, 5 * 37 + 2, 1] = (cand[0, 5 * 37 + 2, 1] + 1) % 400
    dcand = torch.from_numpy(cand).to(device)
    ncand = torch.tensor(sizes, dtype=torch.int32, device=device)
    dcad = torch.from_numpy(np.stack([np.pad(sc[0], ((0, V1 - sc[0].shape[0]), (0, 0))) for sc in scenes])).to(device)
    dpc = torch.from_numpy(np.stack([np.pad(sc[1], ((0, V2 - sc[1].shape[0]), (0, 0))) for sc in scenes])).to(device)
    thr = ops.rigidity_thresholds([sc[3] for sc in scenes], device)
    r0, n0, s0 = _rigid_dev(dl, 0, dcand, ncand, dcad, dpc, thr)
    r3, n3, s3 = _rigid_dev(dl, 3, dcand, ncand, dcad, dpc, thr)
    assert torch.equal(n0, n3)
    assert torch.equal(r0, r3)
    for b in range(len(sizes)):  # the last round's scores over its input list (the round-2 survivors)
        assert torch.equal(s0[b].view(torch.int32), s3[b].view(torch.int32)), b
    assert int(n0.sum()) > 0


@pytest.mark.parametrize("order", ["shuffled", "one_split_group"])
def test_rigidity_filter_candidate_orders(device, order):
    """The first round shares one crop distance per pair of 5-candidate groups (nn_query's
    pc-major order, spacial_filtering.py:36-38); candidate lists in another order take the
    general pair form tile by tile. Shuffled: every tile general; one split group: one group's
    members point at two crop points, so only the tile pairs touching it are general."""
    from dpfm_amd import ops
    cad, pc, cand, diam = _rigid_scene(400, 23)
    cand = cand.copy()
    if order == "shuffled":
        cand = cand[np.random.default_rng(5).permutation(cand.shape[0])]
    else:
        cand[5 * 37 + 2, 1] = (cand[5 * 37 + 2, 1] + 1) % 400
    thr = ops.rigidity_thresholds([diam], device)
    rows, n = ops.rigidity_filter(torch.from_numpy(cand)[None].to(device),
                                  torch.tensor([cand.shape[0]], dtype=torch.int32, device=device),
                                  torch.from_numpy(cad)[None].to(device), torch.from_numpy(pc)[None].to(device), thr)
    _rigidity_parity(cad, pc, cand, rows[0].cpu().numpy(), int(n[0]), diam)


def test_ransac_configs4(device, coracle):
    """configs[4]'s pose stage: 1024 hypotheses over n = 4096 correspondences (4096-vertex CAD)
    vs the C oracle on the same hash-drawn hypotheses: same best hypothesis and fitness, pose
    within 1e-4 (the north-star tolerance)."""
    from _util import cp
    from dpfm_amd.dataset.synthetic import random_rotation
    from dpfm_amd.pose.ransac import ransac_registration
    rng = np.random.default_rng(44)
    R = random_rotation(rng)
    t = np.array([5.0, -3.0, 95.0])
    V = 4096
    cad = rng.normal(size=(V, 3)) * 6
    perm = rng.permutation(V)                 # crop point j was generated by CAD point perm[j]
    pc = (cad[perm] + rng.normal(size=(V, 3)) * 0.01) @ R.T + t
    src_idx = rng.integers(0, V, V)
    dst_idx = rng.integers(0, V, V)
    good = rng.random(V) < 0.3                # 30 % inliers
    src_idx[good] = perm[dst_idx[good]]
    corres = np.ascontiguousarray(np.stack([src_idx, dst_idx], 1).astype(np.int32))
    H = 1024
    T_c, st_c = np.zeros(16), np.zeros(3)
    coracle.oc_ransac(cp(np.ascontiguousarray(cad)), cp(np.ascontiguousarray(pc)), cp(corres), V, None, 7, H, 0.05,
                      cp(T_c), cp(st_c))
    res = ransac_registration(cad, pc, corres, distance_threshold=0.05, max_iteration=H, seed=7, device=device)
    assert res.best_hypothesis == int(st_c[2]) and res.fitness == st_c[0]
    np.testing.assert_allclose(res.transformation, T_c.reshape(4, 4), atol=1e-4)


@pytest.mark.parametrize("N,checked", [(1024, 32), (2048, 4)])
def test_infer_step_configs1_vs_oracle_chain(device, coracle, N, checked):
    """configs[1] (B = 32 x 1024) and the configs[3] per-rank shard (B = 32 x 2048): InferStep
    vs the per-crop oracle chain, stage by stage (each stage's oracle runs on the device's
    previous-stage output, so a near-tie upstream cannot cascade): C for all 32 crops (3x the
    fp32 reference's error vs fp64); for the first `checked` crops (the CPU oracle's rigidity
    rounds at n = 10240 take seconds per crop): top-5, rigidity survivors (exact unless an
    oracle score lies within 1e-5 of its threshold, counted), IR (exact), RANSAC (C oracle, same
    draws: best hypothesis, fitness, pose within 1e-4), pose metrics."""
    from _util import cp
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import InferStep, make_frame_batch, model_batch
    B, H = 32, 1024
    fb, op = make_frame_batch(B, N, N, seed=300, device=device)
    crops = CropFormation(n1=N, npoint=N, seed=9)(fb)
    torch.manual_seed(11)
    ref = M.DPFMNet()
    mine = DPFMNet().to(device)
    mine.load_state_dict(ref.state_dict())
    out = InferStep(mine, hypotheses=H, seed=5)(fb, op, crops)
    torch.cuda.synchronize()
    # (1) the model's C vs the oracle in fp64 / fp32 on the same padded batch
    mb = model_batch(op, crops)
    cpu = {k: {kk: vv.cpu() for kk, vv in v.items() if kk in ("xyz", "mass", "evals", "evecs")} for k, v in mb.items()}
    with torch.no_grad():
        C32 = ref(cpu)[0]
        truth = M.DPFMNet().double()
        truth.load_state_dict(ref.state_dict())
        C64 = truth({k: {kk: vv.double() for kk, vv in v.items()} for k, v in cpu.items()})[0]
    Cg = out["C"].cpu().double()
    e_ref = (C32.double() - C64).abs().max().item()
    assert (Cg - C64).abs().max().item() <= 3 * e_ref + 1e-6 * (1 + C64.abs().max().item())
    cand = out["cand"].cpu().numpy()
    p_pred = out["p_pred"].cpu().numpy()
    ncorr = out["n_corr"].cpu().numpy()
    ir = out["ir"].cpu().numpy()
    T = out["T"].cpu().numpy()
    st = out["ransac"].cpu().numpy()
    ex, ey = cpu["shape1"]["evecs"], cpu["shape2"]["evecs"]
    cadx, pcx, al = cpu["shape1"]["xyz"], cpu["shape2"]["xyz"], crops.align32.cpu()
    cad64 = fb.cad64.cpu().numpy()
    pc64 = crops.pc64.cpu().numpy()
    off = crops.off.cpu().numpy()
    diam = fb.diam
    ties = 0
    for b in range(checked):
        # (2) top-5 on the device's C
        dist = torch.cdist(ex[b, :, :30] @ out["C"][b].cpu().t(), ey[b, :, :30]).numpy().astype(np.float64)
        ties += check_topk(dist, cand[b, :, 0].reshape(N, 5), 5)
        # (3) rigidity filter on the device's candidates, near-threshold scores counted
        surv = p_pred[b, :ncorr[b]]
        _rigidity_parity(cadx[b], pcx[b], cand[b], None, 0, diam[b], got=surv)
        # (4) IR of the device's survivors (eval.py:89)
        exp_ir = O.compute_inlier_ratio(torch.from_numpy(surv), cadx[b], al[b], np.float32(0.1 * diam[b]))
        assert float(ir[b]) == float(exp_ir), b
        # (5) RANSAC on the device's survivors, same hypotheses
        cad_b = np.ascontiguousarray(cad64[N * b:N * (b + 1)])
        pc_b = np.ascontiguousarray(pc64[off[b]:off[b + 1]])
        cor = np.ascontiguousarray(surv.astype(np.int32))
        T_c, st_c = np.zeros(16), np.zeros(3)
        coracle.oc_ransac(cp(cad_b), cp(pc_b), cp(cor), int(ncorr[b]), None, 5, H, 0.05, cp(T_c), cp(st_c))
        assert int(st[b, 2]) == int(st_c[2]) and st[b, 0] == st_c[0], b
        np.testing.assert_allclose(T[b], T_c.reshape(4, 4), atol=1e-4)
        # (6) ADD of the device's pose (test_RANSAC.py:162-173)
        T_gt = np.eye(4)
        T_gt[:3, :3] = fb.R[b].cpu().numpy().reshape(3, 3)
        T_gt[:3, 3] = fb.t[b].cpu().numpy()
        e_add, _ = O.add(T[b], T_gt, cad_b, diam[b])
        np.testing.assert_allclose(out["metrics"][b, 0].item(), e_add, rtol=1e-9)
    assert ties <= checked * N // 200, ties


def test_train_step_configs2_vs_oracle(device):
    """configs[2]'s per-rank step at configs[1]'s shape (B = 32 crops x 1024 points): one
    TrainStep.forward_backward (fused encoder, NCE on the device draw, grouped weight
    gradients) vs the reference training step restated by the oracle (utils/utils.py:67-79
    C_gt, utils/loss.py DPFMLoss, autograd) evaluated in fp64 (the truth), with the same
    weights, crops and NCE pair draw; bars in _util.train_step_parity."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.pipeline import make_frame_batch
    B, N = 32, 1024
    fb, op = make_frame_batch(B, N, N, seed=600, device=device)
    crops = CropFormation(n1=N, npoint=N, seed=4)(fb)
    assert int(crops.npairs.min()) > 0
    train_step_parity(M, op, crops, device, model_seed=21, step_seed=13)


@pytest.mark.parametrize("precision", ["bf16", "bf16x3"])
def test_feat_dist_bf16_configs4_and_ransac(device, coracle, precision):
    """configs[4] as BASELINE.json names it: the 4096 x 4096 feature distance on the bf16 MFMA
    (opt-in precisions; the fp32 path is the parity path) + 1024-hypothesis RANSAC on its
    output. bf16: first choices agree with torch.cdist's argmin on >= 99 % of the columns and
    every pick is within the bf16 rounding band (1e-2 of the largest distance) of the true
    minimum; bf16x3 (hi.hi + hi.lo + lo.hi): exact except near-ties within 1e-4 of the largest
    distance (counted). RANSAC over the bf16 correspondences vs the C oracle on the same
    hypotheses: same best hypothesis and fitness, pose within 1e-4."""
    from _util import cp
    from dpfm_amd import ops
    from dpfm_amd.dataset.synthetic import random_rotation
    from dpfm_amd.pose.ransac import ransac_registration
    V = 4096
    rng = np.random.default_rng(4096)
    ex = _spectral(V, 404)
    perm = rng.permutation(V)                      # crop point j <-> CAD point perm[j]
    ey = ex[perm] + 0.002 * torch.from_numpy(rng.normal(size=(V, ex.shape[1]))).float()
    C = torch.eye(30) + 0.01 * torch.from_numpy(rng.normal(size=(30, 30))).float()
    n = torch.full((1,), V, dtype=torch.int32, device=device)
    i1, _ = ops.feat_dist_topk(ex[None].to(device), C[None].to(device), ey[None].to(device), n, n, 1,
                               precision=precision)
    got = i1[0, :, 0].cpu().numpy()
    dist = torch.cdist(ex[:, :30] @ C.t(), ey[:, :30]).numpy().astype(np.float64)
    best = dist.min(0)
    exp = np.argmin(dist, axis=0)
    picked = dist[got, np.arange(V)]
    agree = float((got == exp).mean())
    if precision == "bf16":
        assert agree >= 0.99, agree
        assert (picked - best <= 1e-2 * dist.max()).all(), float((picked - best).max())
    else:
        ties = check_topk(dist, got[:, None], 1, rel=1e-4)
        assert ties <= V // 1000, ties
    # RANSAC (test_RANSAC.py:288-310) over the correspondences (CAD idx, crop idx)
    R = random_rotation(rng)
    t = np.array([4.0, -2.0, 88.0])
    cad = rng.normal(size=(V, 3)) * 6
    pc = (cad[perm] + rng.normal(size=(V, 3)) * 0.01) @ R.T + t
    corres = np.ascontiguousarray(np.stack([got, np.arange(V)], 1).astype(np.int32))
    H = 1024
    T_c, st_c = np.zeros(16), np.zeros(3)
    coracle.oc_ransac(cp(np.ascontiguousarray(cad)), cp(np.ascontiguousarray(pc)), cp(corres), V, None, 3, H, 0.05,
                      cp(T_c), cp(st_c))
    res = ransac_registration(cad, pc, corres, distance_threshold=0.05, max_iteration=H, seed=3, device=device)
    assert res.best_hypothesis == int(st_c[2]) and res.fitness == st_c[0]
    np.testing.assert_allclose(res.transformation, T_c.reshape(4, 4), atol=1e-4)
    assert res.fitness >= 0.5 * agree  # the recovered pose explains the matched points


@pytest.mark.parametrize("B,V,ragged", [(4, 1024, False), (32, 256, False), (6, 1024, True)])
def test_feat_dist_top5_exact_vs_emulated_chain(device, B, V, ragged):
    """The round-6 top-5 pass (stream minima + candidate lists + exact recomputation) against the
    host emulation of the same fp32 distances (tests/_util.fd_emulate: the prep's operands and
    the MFMA's fmaf chain) and their stable order: indices, and distances as the sqrt of the
    clamped values. Row parts (B = 4: RS = 4 + the merge launch), one part per block (B = 32 x 256),
    ragged crops with fewer than 5 CAD rows (-1 entries) and empty columns. At most one column per
    case may differ, by a double rounding of the host's float64 fmaf emulation."""
    from dpfm_amd import ops
    from _util import fd_emulate, fd_expected_topk
    g = torch.Generator().manual_seed(B * 7 + V)
    ex = torch.stack([_spectral(V, 300 + b) for b in range(B)])
    ey = torch.stack([_spectral(V, 400 + b) for b in range(B)])
    C = torch.eye(30)[None] + 0.3 * torch.randn(B, 30, 30, generator=g)
    if ragged:
        n1 = [3, 5, 17, 300, 1000, V][:B]
        n2 = [V, 40, 1, 513, 999, 7][:B]
    else:
        n1 = n2 = [V] * B
    t1 = torch.tensor(n1, dtype=torch.int32, device=device)
    t2 = torch.tensor(n2, dtype=torch.int32, device=device)
    idx, dist = ops.feat_dist_topk(ex.to(device), C.to(device), ey.to(device), t1, t2, 5, want_dist=True)
    i1, d1 = ops.feat_dist_topk(ex.to(device), C.to(device), ey.to(device), t1, t2, 1, want_dist=True)
    idx, dist, i1, d1 = idx.cpu().numpy(), dist.cpu().numpy(), i1.cpu().numpy(), d1.cpu().numpy()
    bad = bad1 = 0
    for b in range(B):
        d = fd_emulate(ex[b].numpy(), C[b].numpy(), ey[b].numpy(), n1[b], n2[b])
        ei, ev = fd_expected_topk(d, 5)
        gi = idx[b, :n2[b]]
        diff = (gi != ei).any(1)
        bad += int(diff.sum())
        ok = ~diff
        np.testing.assert_array_equal(dist[b, :n2[b]][ok], np.sqrt(ev)[ok])
        # the top-1 pass on the same operands: the first of the five
        d1ff = i1[b, :n2[b], 0] != ei[:, 0]
        bad1 += int(d1ff.sum())
        np.testing.assert_array_equal(d1[b, :n2[b], 0][~d1ff], np.sqrt(ev[:, 0])[~d1ff])
    assert bad <= 1 and bad1 <= 1, (bad, bad1)


def test_feat_dist_top5_duplicates_and_clamp(device):
    """Exact ties and torch.cdist's clamp: crop features equal to CAD rows (C = I) give distances at
    or below 1e-30 (clamped, so tied), and each such CAD row is duplicated at a later row: the five
    must list the tied rows lowest first, then the rest in order (the slow path of the top-5 pass),
    with and without row parts."""
    from dpfm_amd import ops
    from _util import fd_emulate, fd_expected_topk
    for B, V in [(2, 1024), (32, 256)]:
        g = torch.Generator().manual_seed(V)
        ex = torch.randn(B, V, 32, generator=g)
        ey = torch.randn(B, V, 32, generator=g)
        C = torch.eye(30).repeat(B, 1, 1)
        for b in range(B):
            src = torch.randperm(V // 2, generator=g)[:20]
            dup = V // 2 + torch.randperm(V // 2, generator=g)[:20]
            ex[b, dup] = ex[b, src]
            ex[b, dup[:10] - 1] = ex[b, src[:10]]  # a third copy for half of them
            cols = torch.randperm(V, generator=g)[:20]
            ey[b, cols] = ex[b, src]
        n = torch.full((B,), V, dtype=torch.int32, device=device)
        idx, dist = ops.feat_dist_topk(ex.to(device), C.to(device), ey.to(device), n, n, 5, want_dist=True)
        idx = idx.cpu().numpy()
        bad = 0
        for b in range(B):
            d = fd_emulate(ex[b].numpy(), C[b].numpy(), ey[b].numpy(), V, V)
            ei, _ = fd_expected_topk(d, 5)
            bad += int((idx[b] != ei).any(1).sum())
        assert bad <= 1, (B, V, bad)
