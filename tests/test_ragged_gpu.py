"""GPU parity on ragged crops — the reference's real case (crops of 200-2000
points, CADs of ~5000 vertices, collate's zero padding, dataset/helpers.py:22-50).

  * CropFormation with the reference's sample policy (npoint = 0) and with a fixed target
    larger than some crops, against the oracle chain per crop (object.py:133-180) followed by
    the oracle's collate: padded PC xyz / align_pc / overlaps bit-exact, pair lists exact.
  * Real crops of the reference's published results (tests/golden/real_crops.npz: camera-
    frame crops pc_i.ply, T_gt, decimated CADs of 4996-5002 vertices): find_positives and
    the inlier ratio bit-exact, DPFMNet forward + gradients on the padded N1 ~ 5000 != N2
    batch within 3x the fp32 reference's own error vs fp64, and a training / inference step.
"""
import os

import numpy as np
import pytest
import torch

from oracle import dpfm_oracle as O
from oracle import dpfm_model_oracle as M

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _frames(seed=0):
    """LM sample frame masks (incl. the empty mask 1 and the tiny mask 14) + synthetic frames,
    each with a pose and a CAD of its own size that overlaps the crop."""
    from dpfm_amd.dataset.synthetic import make_frame, random_rotation
    g = np.load(os.path.join(GOLD, "lm_frame.npz"))
    rng = np.random.default_rng(seed)
    raw = [(g["depth"], g["masks"][j], g["K"], float(g["depth_scale"])) for j in range(g["masks"].shape[0])]
    for s in range(3):
        f = make_frame(100 + s)
        raw.append((f.depth, f.mask, f.K, f.depth_scale))
    frames = []
    for b, (depth, mask, K, ds) in enumerate(raw):
        R = random_rotation(rng)
        t = rng.normal(size=3) * 20 + np.array([0, 0, 90.0])
        pts = O.dpt_2_pcld(depth, 1000 / ds, K, mask == 255)
        n1 = 300 + 37 * b
        if pts.shape[0]:
            src = O.transform(pts[rng.integers(0, pts.shape[0], n1)], R, t, inv=True)
            cad = src + rng.normal(size=src.shape) * 0.4
        else:
            cad = rng.normal(size=(n1, 3)) * 5
        frames.append(dict(depth=depth, mask=mask, K=K, depth_scale=ds, R_m2c=R, t_m2c=t, cad=cad,
                           diam_cad=12.0 + b))
    return frames


def _oracle_items(frames, seed, fixed):
    items = []
    for b, f in enumerate(frames):
        pcd = O.remove_outliers(O.dpt_2_pcld(f["depth"], 1000 / f["depth_scale"], f["K"], f["mask"] == 255))
        pcd = O.sample_crop(pcd, seed, b, fixed=fixed)
        align = O.transform(pcd, f["R_m2c"], f["t_m2c"], inv=True)
        P = O.find_positives(f["cad"], align, r=f["diam_cad"] * 0.05)
        o12, o21 = O.get_overlap(f["cad"].shape[0], pcd.shape[0], P)
        items.append(({"xyz": f["cad"]}, {"xyz": pcd.astype(np.float32)},
                      {"align_pc": align, "P": P, "overlap_12": o12, "overlap_21": o21, "obj_id": b}))
    return items


@pytest.mark.parametrize("fixed", [0, 1024])
def test_crop_formation_ragged_matches_collate(device, fixed):
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.pipeline import frame_batch
    frames = _frames()
    seed = 11
    fb = frame_batch(frames, device)
    crops = CropFormation(npoint=fixed, seed=seed, pad="batch")(fb)
    items = _oracle_items(frames, seed, fixed)
    CAD, PC, Obj = O.collate(items)
    n2 = [it[1]["xyz"].shape[0] for it in items]
    assert crops.n2.cpu().tolist() == n2
    assert crops.ld == max(n2) and PC["xyz"].shape[1] == crops.ld
    assert 0 in n2 and any(0 < n < 1024 for n in n2)  # an empty and a small crop
    if fixed == 0:
        assert max(n2) in (1999, 2000) and any(1024 < n < 1999 for n in n2)
    else:
        assert max(n2) == fixed
    assert torch.equal(crops.pc32.cpu(), PC["xyz"])              # PC["xyz"]: f32, zero-padded
    assert torch.equal(crops.align32.cpu(), Obj["align_pc"])     # Obj["align_pc"]
    assert torch.equal(crops.overlap_21.cpu().float(), Obj["overlap_21"])
    assert torch.equal(crops.overlap_12.cpu().float(), Obj["overlap_12"])
    npairs = crops.npairs.cpu().numpy()
    pairs = crops.pairs.cpu().numpy()
    for b, P in enumerate(Obj["P"]):
        assert npairs[b] == P.shape[0], b
        np.testing.assert_array_equal(pairs[b, :npairs[b]], P.numpy().astype(np.int64))
    assert not bool(crops.overflow())
    # packed camera-frame crops (RANSAC's target) equal the oracle's f64 points
    off = crops.off.cpu().numpy()
    pc64 = crops.pc64.cpu().numpy()
    for b, it in enumerate(items):
        np.testing.assert_array_equal(pc64[off[b]:off[b + 1]].astype(np.float32), it[1]["xyz"])


def test_pair_capacity_overflow_is_flagged(device):
    from dpfm_amd import ops
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.pipeline import frame_batch
    frames = _frames()[:4]
    crops = CropFormation(npoint=0, seed=3, pad="batch", pair_cap=8)(frame_batch(frames, device))
    assert bool(crops.overflow())
    with pytest.raises(ops._lib.PoseKernError):
        crops.check()


def test_train_step_on_ragged_crops(device):
    """A training step over ragged crops (LM masks + synthetic frames: 0- to 2000-point crops,
    collate padding): finite loss, no pair overflow, IR in [0, 1], parameters updated; and the
    same step's forward_backward vs the oracle's training step in fp64 (C_gt, loss, every
    parameter gradient; bars of _util.train_step_parity) on the padded ragged batch."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import TrainStep, frame_batch, operators_for
    from _util import train_step_parity
    frames = [f for f in _frames() if f["mask"].any()][:6]
    fb = frame_batch(frames, device)
    crops = CropFormation(npoint=0, seed=5, pad="batch")(fb)
    op = operators_for([f["cad"] for f in frames], crops.n2.cpu().tolist(), fb.diam, 0, device, ld2=crops.ld)
    assert crops.ld >= 1999 and min(crops.n2.cpu().tolist()) < 1024
    torch.manual_seed(0)
    model = DPFMNet().to(device)
    step = TrainStep(model)
    before = [p.detach().clone() for p in model.parameters()]
    log = step(op, crops)
    torch.cuda.synchronize()
    assert np.isfinite(float(log["loss"])) and not bool(log["pair_overflow"])
    assert 0.0 <= float(log["IR"]) <= 1.0
    assert any(not torch.equal(a, p) for a, p in zip(before, model.parameters()))
    train_step_parity(M, op, crops, device, model_seed=17, step_seed=29)


# ----------------------------------------------------------------------------- real crops


def _real():
    g = np.load(os.path.join(GOLD, "real_crops.npz"))
    out = []
    for k in range(int(g["n"])):
        T = g[f"{k}_T_gt"]
        oid = int(g[f"{k}_obj_id"])
        out.append(dict(pc=g[f"{k}_pc"], R=T[:3, :3].copy(), t=T[:3, 3].copy(), cad=g[f"cad_{oid}"],
                        diam=float(g[f"{k}_diam"]), obj_id=oid))
    return out


def test_real_crops_find_positives_and_ir(device):
    """object.py:174-180 on the reference's own crops and CADs: align_pc (H4) in the
    oracle's evaluation order, the ball query (H5) and overlaps bit-exact; the inlier ratio
    (H12) of the pair list exact."""
    from dpfm_amd import ops
    crops = _real()
    B = len(crops)
    align = [O.transform(c["pc"], c["R"], c["t"], inv=True) for c in crops]
    cad = torch.from_numpy(np.concatenate([c["cad"] for c in crops])).to(device)
    cad_off = ops.packed_offsets([c["cad"].shape[0] for c in crops], device)
    # H4 on the device (gather_transform with every point kept)
    pcs = torch.from_numpy(np.concatenate([c["pc"] for c in crops])).to(device)
    pc_off = ops.packed_offsets([c["pc"].shape[0] for c in crops], device)
    n2 = [c["pc"].shape[0] for c in crops]
    npoint = torch.tensor([-n for n in n2], dtype=torch.int32, device=device)
    R = torch.from_numpy(np.stack([c["R"].reshape(9) for c in crops])).to(device)
    t = torch.from_numpy(np.stack([c["t"] for c in crops])).to(device)
    g = ops.gather_transform(pcs, pc_off, None, npoint, max(n2), pc_off, R, t, sum(n2), want_sel32=False)
    np.testing.assert_array_equal(g["align"].cpu().numpy(), np.concatenate(align))
    n1max = max(c["cad"].shape[0] for c in crops)
    res = ops.ball_query(cad, cad_off, g["align"], pc_off, [0.05 * c["diam"] for c in crops], n1max, max(n2), 1 << 20)
    cnt = res["count"].cpu().numpy()
    pairs = res["pairs"].cpu().numpy()
    o12 = res["overlap_12"].cpu().numpy()
    o21 = res["overlap_21"].cpu().numpy()
    cad32 = torch.zeros((B, n1max, 3), dtype=torch.float32)
    al32 = torch.zeros((B, max(n2), 3), dtype=torch.float32)
    for b, c in enumerate(crops):
        P = O.find_positives(c["cad"], align[b], r=c["diam"] * 0.05)
        assert P.shape[0] > 0
        assert cnt[b] == P.shape[0], b
        np.testing.assert_array_equal(pairs[b, :cnt[b]], P)
        e12, e21 = O.get_overlap(c["cad"].shape[0], n2[b], P)
        np.testing.assert_array_equal(o12[b, :e12.shape[0]], e12)
        np.testing.assert_array_equal(o21[b, :n2[b]], e21)
        cad32[b, :c["cad"].shape[0]] = torch.Tensor(c["cad"])
        al32[b, :n2[b]] = torch.Tensor(align[b])
    # IR of a correspondence set mixing true pairs and shuffled ones (utils/utils.py:81-105)
    rng = np.random.default_rng(0)
    L = 600
    corr = np.zeros((B, L, 2), dtype=np.int64)
    ncorr = []
    exp = []
    for b, c in enumerate(crops):
        P = pairs[b, :cnt[b]]
        m = min(L, 100 + 50 * b)
        sel = P[rng.integers(0, P.shape[0], m)].copy()
        sel[::3, 0] = rng.integers(0, c["cad"].shape[0], sel[::3].shape[0])
        corr[b, :m] = sel
        ncorr.append(m)
        exp.append(float(O.compute_inlier_ratio(torch.from_numpy(sel), cad32[b], al32[b],
                                                np.float32(0.1 * c["diam"]))))
    thr = torch.tensor([np.float32(0.1 * c["diam"]) for c in crops], device=device)
    ir = ops.inlier_ratio(torch.from_numpy(corr).to(device), torch.tensor(ncorr, dtype=torch.int32, device=device),
                          cad32.to(device), al32.to(device), thr, layout=0).cpu().numpy()
    np.testing.assert_array_equal(ir, np.asarray(exp, dtype=np.float32))


def _real_batch(idx, seed=0):
    """collate of the chosen real crops with synthetic operators of the true sizes."""
    from dpfm_amd.pipeline import lbo_padded
    crops = [_real()[i] for i in idx]
    items = []
    for b, c in enumerate(crops):
        cm, ce, cv = lbo_padded(c["cad"].shape[0], 2 * (seed + b))
        pm, pe, pv = lbo_padded(c["pc"].shape[0], 2 * (seed + b) + 1)
        items.append(({"xyz": c["cad"], "mass": cm, "evals": ce, "evecs": cv},
                      {"xyz": c["pc"].astype(np.float32), "mass": pm, "evals": pe, "evecs": pv}, {"obj_id": 0}))
    CAD, PC, _ = O.collate(items)
    return crops, {"shape1": CAD, "shape2": PC}


def test_dpfmnet_real_crops_matches_oracle(device):
    """DPFMNet forward + parameter gradients on a padded batch of real crops (N1 = 5002, N2 =
    2000 with 200- and 1821-point crops padded) vs the oracle in fp64; bar: 3x the larger
    error of the fp32 reference on the CPU and torch on the GPU (test_model_gpu's yardstick)."""
    from dpfm_amd.models.dpfm import DPFMNet
    from _util import model_parity
    _, batch = _real_batch([0, 3, 6])
    assert batch["shape1"]["xyz"].shape[1] == 5002 and batch["shape2"]["xyz"].shape[1] == 2000
    torch.manual_seed(7)
    model_parity(M, DPFMNet, batch, device)


def test_infer_step_on_real_crops(device, coracle):
    """Inference (eval.py + test_RANSAC.py) on the reference's real crops (200-2000 points,
    ~5000-vertex CADs): the spatial-filter solver on the non-padding rows, RANSAC in the camera
    frame, checked stage by stage against the oracle chain (below)."""
    from dpfm_amd import ops
    from dpfm_amd.dataset.object import Crops, FrameBatch
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import InferStep, model_batch, operators_for
    from _util import check_topk, cp, rigidity_parity
    crops_np = _real()
    B = len(crops_np)
    n2 = [c["pc"].shape[0] for c in crops_np]
    ld = max(n2)
    op = operators_for([c["cad"] for c in crops_np], n2, [c["diam"] for c in crops_np], 0, device, ld2=ld)
    pc_off = ops.packed_offsets(n2, device)
    pc64 = torch.from_numpy(np.concatenate([c["pc"] for c in crops_np])).to(device)
    pc32, n2t = ops.collate_pad(pc64, pc_off, ld)
    al = torch.from_numpy(np.concatenate([O.transform(c["pc"], c["R"], c["t"], inv=True) for c in crops_np]))
    al32, _ = ops.collate_pad(al.to(device), pc_off, ld)
    cads = [c["cad"] for c in crops_np]
    cad_off = ops.packed_offsets([len(c) for c in cads], device)
    fb = FrameBatch(depth=None, mask=None, rgb=None, K=None, cam_scale=None,
                    R=torch.from_numpy(np.stack([c["R"].reshape(9) for c in crops_np])).to(device),
                    t=torch.from_numpy(np.stack([c["t"] for c in crops_np])).to(device),
                    cad64=torch.from_numpy(np.concatenate(cads)).to(device), cad_off=cad_off,
                    diam=[c["diam"] for c in crops_np], max_pixels=0, thr2=None, n1max=max(len(c) for c in cads))
    crops = Crops(pc64=pc64, pc32=pc32, align64=al.to(device), align32=al32, off=pc_off, n2=n2t, ld=ld, npoint=None,
                  pairs=None, npairs=None, overlap_12=None, overlap_21=None, rgb=None, kept=None)
    torch.manual_seed(1)
    ref = M.DPFMNet()
    mine = DPFMNet().to(device)
    mine.load_state_dict(ref.state_dict())
    H = 256
    res = InferStep(mine, hypotheses=H, seed=3)(fb, op, crops)
    torch.cuda.synchronize()
    assert torch.isfinite(res["T"]).all() and torch.isfinite(res["metrics"]).all()
    ncorr = res["n_corr"].cpu().numpy()
    assert (ncorr >= 0).all() and (ncorr <= 5 * np.asarray(n2)).all()
    ir = res["ir"].cpu().numpy()
    assert ((ir >= 0) & (ir <= 1)).all()
    # stage by stage vs the oracle chain (each stage's oracle on the device's previous-stage
    # output, as test_configs_gpu.py::test_infer_step_configs1_vs_oracle_chain): the model's C on
    # the padded 5002 x 2000 batch, then for two crops (200 and ~1000 points; the CPU oracle's
    # rigidity rounds are O(n^2) at n = 5 n2) top-5 on the valid rows, rigidity survivors, IR,
    # RANSAC (C oracle, same draws) and ADD.
    mb = model_batch(op, crops)
    cpu = {k: {kk: vv.cpu() for kk, vv in v.items() if kk in ("xyz", "mass", "evals", "evecs")} for k, v in mb.items()}
    with torch.no_grad():
        C32 = ref(cpu)[0]
        truth = M.DPFMNet().double()
        truth.load_state_dict(ref.state_dict())
        C64 = truth({k: {kk: vv.double() for kk, vv in v.items()} for k, v in cpu.items()})[0]
    Cg = res["C"].cpu().double()
    e_ref = (C32.double() - C64).abs().max().item()
    assert (Cg - C64).abs().max().item() <= 3 * e_ref + 1e-6 * (1 + C64.abs().max().item())
    cand = res["cand"].cpu().numpy()
    p_pred = res["p_pred"].cpu().numpy()
    T = res["T"].cpu().numpy()
    st = res["ransac"].cpu().numpy()
    ex, ey = cpu["shape1"]["evecs"], cpu["shape2"]["evecs"]
    cadx, pcx, al32c = cpu["shape1"]["xyz"], cpu["shape2"]["xyz"], crops.align32.cpu()
    order = np.argsort(n2)
    ties = 0
    for b in (int(order[0]), int(order[len(order) // 2])):
        n1b, n2b = cads[b].shape[0], n2[b]
        dist = torch.cdist(ex[b, :n1b, :30] @ res["C"][b].cpu().t(), ey[b, :n2b, :30]).numpy().astype(np.float64)
        ties += check_topk(dist, cand[b, :5 * n2b, 0].reshape(n2b, 5), 5)
        surv = p_pred[b, :ncorr[b]]
        rigidity_parity(cadx[b, :n1b], pcx[b, :n2b], cand[b, :5 * n2b], None, 0, crops_np[b]["diam"], got=surv)
        exp_ir = O.compute_inlier_ratio(torch.from_numpy(surv), cadx[b], al32c[b], np.float32(0.1 * crops_np[b]["diam"]))
        assert float(ir[b]) == float(exp_ir), b
        cor = np.ascontiguousarray(surv.astype(np.int32))
        T_c, st_c = np.zeros(16), np.zeros(3)
        coracle.oc_ransac(cp(np.ascontiguousarray(cads[b])), cp(np.ascontiguousarray(crops_np[b]["pc"])), cp(cor),
                          int(ncorr[b]), None, 3, H, 0.05, cp(T_c), cp(st_c))
        assert int(st[b, 2]) == int(st_c[2]) and st[b, 0] == st_c[0], b
        np.testing.assert_allclose(T[b], T_c.reshape(4, 4), atol=1e-4)
        T_gt = np.eye(4)
        T_gt[:3, :3], T_gt[:3, 3] = crops_np[b]["R"], crops_np[b]["t"]
        e_add, _ = O.add(T[b], T_gt, cads[b], crops_np[b]["diam"])
        np.testing.assert_allclose(res["metrics"][b, 0].item(), e_add, rtol=1e-9)
    assert ties <= max(2, (n2[int(order[0])] + n2[int(order[len(order) // 2])]) // 200), ties


def test_cgt_real_crops_full_rank(device):
    """C_from_sparse_P (utils/utils.py:67-79) on the pair lists of the reference's own crops
    (find_positives on tests/golden/real_crops.npz: 5000-vertex CADs, 200-2000-point crops) with
    operator stand-ins of the true sizes: full-rank systems, where the reference's GPU `gels` and
    the CPU drivers agree, so this is the pinned case of pk_cgt_lstsq (the rank-deficient
    min-norm path is a documented deviation). fp32 device result within 1e-4 of the fp64 oracle's
    scale."""
    from dpfm_amd import ops
    from dpfm_amd.pipeline import lbo_padded
    crops = _real()
    B = len(crops)
    n1 = [c["cad"].shape[0] for c in crops]
    n2 = [c["pc"].shape[0] for c in crops]
    plist = []
    for c in crops:
        align = O.transform(c["pc"], c["R"], c["t"], inv=True)
        plist.append(torch.from_numpy(O.find_positives(c["cad"], align, r=c["diam"] * 0.05)))
    cap = max(p.shape[0] for p in plist)
    pairs = torch.zeros((B, cap, 2), dtype=torch.int64)
    for b, p in enumerate(plist):
        pairs[b, :p.shape[0]] = p
    e1 = torch.zeros((B, max(n1), 64))
    e2 = torch.zeros((B, max(n2), 64))
    for b in range(B):
        e1[b, :n1[b]] = torch.from_numpy(lbo_padded(n1[b], 2 * b)[2])
        e2[b, :n2[b]] = torch.from_numpy(lbo_padded(n2[b], 2 * b + 1)[2])
    got = ops.cgt_lstsq(pairs.to(device), torch.tensor([p.shape[0] for p in plist], device=device), e1.to(device),
                        e2.to(device)).cpu().double()
    for b, p in enumerate(plist):
        assert len(set(p[:, 1].tolist())) >= 30  # full rank: at least 30 distinct crop rows
        exp = M.C_from_sparse_P(p, e1[b, :n1[b], :30].double(), e2[b, :n2[b], :30].double())
        scale = float(exp.abs().max())
        assert (got[b] - exp).abs().max().item() <= 1e-4 * scale, (b, (got[b] - exp).abs().max().item(), scale)


def test_cgt_real_crops_full_rank_fp32_oracle(device):
    """C_from_sparse_P (utils/utils.py:67-79) on the reference's own pair structure: the ball-query
    positives of its real crops (object.py:174-177, r = 0.05 diam) with operators of the true
    sizes. Every crop matches >= 30 distinct crop rows, so the normal equations are full rank and
    pk_cgt_lstsq takes its Gauss-Jordan path; C_gt agrees with the torch lstsq restatement
    (fp32 tolerance of the 30 x 30 solve). The rank-deficient / empty cases, where the device
    returns the minimum-norm solution, are test_corr_pose_gpu.py::test_cgt_rank_deficient_and_empty."""
    from dpfm_amd import ops
    from dpfm_amd.pipeline import lbo_padded
    crops = _real()
    B = len(crops)
    Ps = [O.find_positives(c["cad"], O.transform(c["pc"], c["R"], c["t"], inv=True), r=c["diam"] * 0.05)
          for c in crops]
    L = max(P.shape[0] for P in Ps)
    V1 = max(c["cad"].shape[0] for c in crops)
    V2 = max(c["pc"].shape[0] for c in crops)
    pairs = np.zeros((B, L, 2), dtype=np.int64)
    e1 = np.zeros((B, V1, 64), dtype=np.float32)
    e2 = np.zeros((B, V2, 64), dtype=np.float32)
    for b, (c, P) in enumerate(zip(crops, Ps)):
        assert np.unique(P[:, 1]).shape[0] >= 30, b  # full rank: >= 30 distinct crop rows
        pairs[b, :P.shape[0]] = P
        e1[b, :c["cad"].shape[0]] = lbo_padded(c["cad"].shape[0], 2 * b)[2]
        e2[b, :c["pc"].shape[0]] = lbo_padded(c["pc"].shape[0], 2 * b + 1)[2]
    got = ops.cgt_lstsq(torch.from_numpy(pairs).to(device),
                        torch.tensor([P.shape[0] for P in Ps], dtype=torch.int64, device=device),
                        torch.from_numpy(e1).to(device), torch.from_numpy(e2).to(device)).cpu()
    for b, P in enumerate(Ps):
        exp = M.C_from_sparse_P(torch.from_numpy(P), torch.from_numpy(e1[b, :, :30]), torch.from_numpy(e2[b, :, :30]))
        scale = max(float(exp.abs().max()), 1e-30)
        torch.testing.assert_close(got[b], exp, rtol=1e-3, atol=1e-4 * scale)
