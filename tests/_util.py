import ctypes

import numpy as np


def cp(a: np.ndarray):
    """ctypes pointer to a contiguous numpy array."""
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def c_fps(coracle, xyz: np.ndarray, start: int, npoint: int) -> np.ndarray:
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    out = np.zeros(npoint, dtype=np.int64)
    coracle.oc_fps(cp(xyz), xyz.shape[0], int(start), int(npoint), cp(out))
    return out


def c_ball_query(coracle, pc1: np.ndarray, pc2: np.ndarray, r: float):
    pc1 = np.ascontiguousarray(pc1, dtype=np.float64)
    pc2 = np.ascontiguousarray(pc2, dtype=np.float64)
    cap = pc1.shape[0] * pc2.shape[0]
    cap = min(cap, 1 << 24)
    pairs = np.zeros((cap, 2), dtype=np.int64)
    o12 = np.zeros(pc1.shape[0], dtype=np.int8)
    o21 = np.zeros(pc2.shape[0], dtype=np.int8)
    n = coracle.oc_ball_query(cp(pc1), pc1.shape[0], cp(pc2), pc2.shape[0], float(r), cp(pairs), cap, cp(o12), cp(o21))
    return pairs[:n], o12, o21


def boundary_cloud(rng, n1: int, n2: int, r: float, scale: float = 8.0, offset=(0.0, 0.0, 110.0)):
    """Two clouds with many pairs at distance ~r (some exactly r up to rounding)."""
    off = np.asarray(offset)
    pc1 = rng.uniform(-scale, scale, size=(n1, 3)) + off
    pick = rng.integers(0, n1, size=n2)
    u = rng.normal(size=(n2, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    jitter = rng.choice([0.0, 1e-15, -1e-15, 1e-9, -1e-9, 0.3, -0.3], size=(n2, 1))
    pc2 = pc1[pick] + u * (r * (1.0 + jitter))
    half = n2 // 2
    pc2[:half] = rng.uniform(-scale, scale, size=(half, 3)) + off
    return pc1, pc2


def model_parity(M, DPFMNet, batch, device, diffusion_times=True):
    """DPFMNet forward outputs and parameter gradients vs the oracle evaluated in fp64 (the
    truth). Yardstick: the same oracle evaluated in fp32 on the CPU (the reference's own
    path) and with torch on the GPU; the HIP path must be within 3x the larger of their
    errors. Gradients are compared as Frobenius norms per parameter, with an absolute floor
    of 1e-6 x the global gradient norm for parameters whose true gradient vanishes by
    invariance (biases in front of InstanceNorm / the softmax's key bias)."""
    import torch
    ref = M.DPFMNet()
    if diffusion_times:
        with torch.no_grad():  # exercise the in-place clamp with negative diffusion times
            ref.feature_extractor.block_0.diffusion.diffusion_time.uniform_(-0.001, 12)
            ref.feature_extractor.block_1.diffusion.diffusion_time.uniform_(-0.001, 12)
    truth = M.DPFMNet().double()
    truth.load_state_dict(ref.state_dict())
    gref = M.DPFMNet().to(device)
    gref.load_state_dict(ref.state_dict())
    mine = DPFMNet().to(device)
    mine.load_state_dict(ref.state_dict(), strict=True)
    to = lambda b, dev: {k: {kk: vv.to(dev) for kk, vv in v.items() if vv is not None} for k, v in b.items()}  # noqa
    batch = {k: {kk: vv for kk, vv in v.items() if vv is not None and kk in ("xyz", "mass", "evals", "evecs")}
             for k, v in batch.items()}
    batch64 = {k: {kk: vv.double() for kk, vv in v.items()} for k, v in batch.items()}
    runs = [(truth, batch64), (ref, batch), (gref, to(batch, device)), (mine, to(batch, device))]
    outs = [m(b) for m, b in runs]
    for n, t, r, g, d in zip(["C", "o12", "o21", "f1", "f2"], *(o[:5] for o in outs)):
        t = t.detach()
        e = [(x.detach().cpu().double() - t).abs().max().item() for x in (r, g, d)]
        assert e[2] <= 3 * max(e[0], e[1]) + 1e-6 * (1 + t.abs().max().item()), (n, e)

    def check(loss_fn, label):
        grads = []
        for m, b in runs:
            m.zero_grad()
            loss_fn(m(b)).backward()
            grads.append([torch.zeros(p.shape, dtype=torch.float64) if p.grad is None else p.grad.detach().cpu().double()
                          for p in m.parameters()])
        floor = 1e-6 * torch.cat([g.reshape(-1) for g in grads[0]]).norm().item()
        for i, (name, _) in enumerate(truth.named_parameters()):
            t = grads[0][i]
            e = [(g[i] - t).norm().item() for g in grads[1:]]
            assert e[2] <= 3 * max(e[0], e[1]) + floor, (label, name, e, floor, t.norm().item())

    check(lambda o: o[1].sum() + o[2].sum() + o[3].square().sum() + o[4].square().sum(), "overlap+features")
    check(lambda o: o[0].sum(), "fmap")


def check_topk(dist: np.ndarray, got: np.ndarray, k: int, rel: float = 1e-5) -> int:
    """dist [V1, V2] (fp64 copy of the oracle's cdist), got [V2, k] row indices. Every column's
    k picks must be distinct and their distances the k smallest of the column in ascending
    order, up to near-ties |d_a - d_b| <= rel * max(d). Returns the number of columns that
    differ from the oracle's stable sort only by such ties."""
    tol = rel * max(float(dist.max()), 1e-12)
    srt = np.sort(dist, axis=0)[:k]                      # [k, V2] the k smallest per column
    picked = np.take_along_axis(dist, got.T, axis=0)     # [k, V2] distances of the picks
    assert (np.abs(picked - srt) <= tol).all(), float(np.abs(picked - srt).max())
    for j in range(got.shape[0]):
        assert len(set(got[j].tolist())) == k, j
    exp = np.argsort(dist, axis=0, kind="stable")[:k].T
    return int((exp != got).any(1).sum())


def rigidity_parity(cad, pc, cand, rows, n, diam, got=None):
    """survivors equal the oracle's on the same candidates, except candidates whose oracle score
    lies within 1e-5 (relative) of its round's threshold. `got`: the device's survivor pairs
    (default cand[rows[:n]])."""
    import torch
    from oracle import dpfm_oracle as O
    cad = cad.numpy() if torch.is_tensor(cad) else cad
    pc = pc.numpy() if torch.is_tensor(pc) else pc
    p = torch.from_numpy(cand).t()
    exp, scores = O.spacial_filtering(torch.from_numpy(cad), torch.from_numpy(pc), p, diam, return_scores=True)
    if got is None:
        got = cand[rows[:n]]
    a, b = set(map(tuple, got.tolist())), set(map(tuple, exp.t().tolist()))
    near = 0
    for s, tau in zip(scores, (0.3, 0.15, 0.055)):
        thr = float(np.float32(tau * diam))
        near += int((np.abs(s.numpy() - thr) <= 1e-5 * thr).sum())
    if near == 0:
        assert a == b and np.array_equal(got, exp.t().numpy())  # same survivors, same order
    else:
        assert len(a ^ b) <= 4 * near + max(2, len(b) // 1000), (len(a ^ b), near)
    return len(b)


def train_step_parity(M, op, crops, device, model_seed, step_seed):
    """One TrainStep.forward_backward (fused encoder, NCE on the device draw, grouped weight
    gradients) vs the reference training step restated by the oracle (utils/utils.py:67-79
    C_gt, utils/loss.py DPFMLoss, autograd) evaluated in fp64 (the truth), with the same
    weights, crops and NCE pair draw. Yardstick (model_parity's): the same oracle in fp32 on
    the CPU and on the GPU; the HIP step's loss and every parameter gradient must be within
    3x the larger of their errors (gradient floor 1e-6 x the global gradient norm for the
    invariance-zero parameters), the oracle's loss taking the step's C_gt; C_gt itself per crop
    within 1e-4 of its scale where the pair system is well conditioned, else a least-squares
    solution at least as good as the fp64 oracle's."""
    import torch
    from dpfm_amd import ops
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import TrainStep, model_batch
    B = crops.npairs.shape[0]
    torch.manual_seed(model_seed)
    ref = M.DPFMNet()
    with torch.no_grad():
        ref.feature_extractor.block_0.diffusion.diffusion_time.uniform_(-0.001, 12)
        ref.feature_extractor.block_1.diffusion.diffusion_time.uniform_(-0.001, 12)
    truth = M.DPFMNet().double()
    truth.load_state_dict(ref.state_dict())
    gref = M.DPFMNet().to(device)
    gref.load_state_dict(ref.state_dict())
    mine = DPFMNet().to(device)
    mine.load_state_dict(ref.state_dict(), strict=True)
    step = TrainStep(mine, seed=step_seed)
    # the step's NCE draw, reproduced from its generator seed and device counter (not advanced)
    cap = crops.pairs.shape[1]
    rows, valid = ops.nce_select(crops.npairs, cap, 512, int(step.gen.initial_seed()), step.nce_counter().clone())
    C_gt_dev = ops.cgt_lstsq(crops.pairs, crops.npairs, op.cad_evecs, op.pc_evecs)
    log = step.forward_backward(op, crops)
    torch.cuda.synchronize()
    npairs = crops.npairs.cpu()
    assert int(npairs.max()) <= cap
    pairs = crops.pairs.cpu()
    plist = [pairs[b, :int(npairs[b])] for b in range(B)]
    sel = [rows[b][valid[b]].cpu() for b in range(B)]
    g12, g21 = crops.overlap_12.cpu(), crops.overlap_21.cpu()
    mb = model_batch(op, crops)
    keys = ("xyz", "mass", "evals", "evecs")
    cpu = {k: {kk: vv.cpu() for kk, vv in v.items() if kk in keys} for k, v in mb.items()}
    cpu64 = {k: {kk: vv.double() for kk, vv in v.items()} for k, v in cpu.items()}
    gpu = {k: {kk: vv.to(device) for kk, vv in v.items()} for k, v in cpu.items()}

    cgd = C_gt_dev.cpu().double()

    def oracle_step(model, batch, dt):
        model.zero_grad()
        ex, ey = batch["shape1"]["evecs"], batch["shape2"]["evecs"]
        C_gt = torch.stack([M.C_from_sparse_P(plist[b].to(ex.device), ex[b, :, :30], ey[b, :, :30]) for b in range(B)])
        if dt == torch.float64:
            C_gt_of[0] = C_gt.detach().cpu().double()
        # the step's own C_gt (checked against this one below, rank-aware): the loss and
        # gradients are then compared on the same target
        C_gt = cgd.to(device=ex.device, dtype=C_gt.dtype)
        C, o12, o21, f1, f2, _, _ = model(batch)
        dv = ex.device
        loss = M.dpfm_loss(C, C_gt, [p.to(dv) for p in plist], [s.to(dv) for s in sel], f1, f2, o12, o21,
                           g12.to(dv), g21.to(dv))
        loss.backward()
        grads = [torch.zeros(p.shape, dtype=torch.float64) if p.grad is None else p.grad.detach().cpu().double()
                 for p in model.parameters()]
        return float(loss), C_gt.detach().cpu().double(), grads

    C_gt_of = [None]
    l64, _, gr64 = oracle_step(truth, cpu64, torch.float64)
    l32, _, gr32 = oracle_step(ref, cpu, torch.float32)
    lg, _, grg = oracle_step(gref, gpu, torch.float32)
    # C_gt per crop: within 1e-4 of its scale where the pair system is well conditioned (>= 30
    # pairs, sigma_min / sigma_max >= 1e-5); otherwise (few or degenerate pairs: the reference's
    # CUDA gels has no defined answer, both sides give a least-squares solution) the device's
    # residual no larger than the fp64 oracle's + 1e-4 of the right-hand side
    cg64 = C_gt_of[0]
    ex64, ey64 = cpu64["shape1"]["evecs"], cpu64["shape2"]["evecs"]
    for b in range(B):
        p = plist[b]
        a1, a2 = ex64[b][p[:, 0], :30], ey64[b][p[:, 1], :30]
        sv = torch.linalg.svdvals(a2) if p.shape[0] else torch.zeros(1, dtype=torch.float64)
        if p.shape[0] >= 30 and float(sv[-1]) >= 1e-5 * float(sv[0]):
            err = (cgd[b] - cg64[b]).abs().max().item()
            assert err <= 1e-4 * max(cg64[b].abs().max().item(), 1e-30), (b, err)
        else:
            rd = (a2 @ cgd[b] - a1).norm().item()
            ro = (a2 @ cg64[b] - a1).norm().item()
            assert rd <= ro + 1e-4 * max(a1.norm().item(), 1e-30), (b, rd, ro)
    # loss
    ld = float(log["loss"])
    e = [abs(l32 - l64), abs(lg - l64), abs(ld - l64)]
    assert e[2] <= 3 * max(e[0], e[1]) + 1e-6 * abs(l64), (e, l64)
    # every parameter gradient
    floor = 1e-6 * torch.cat([g.reshape(-1) for g in gr64]).norm().item()
    mine_g = [p.grad.detach().cpu().double() for p in mine.parameters()]
    for (name, _), t, a, b, d in zip(truth.named_parameters(), gr64, gr32, grg, mine_g):
        ee = [(a - t).norm().item(), (b - t).norm().item(), (d - t).norm().item()]
        assert ee[2] <= 3 * max(ee[0], ee[1]) + floor, (name, ee, floor, t.norm().item())


def fd_emulate(ex, C, ey, n1: int, n2: int):
    """The fp32 feature-distance pass's distances [n1, n2], emulated on the host: the prep's -2 emb
    = -2 x C^T and |emb|^2, the columns' [y, 1, |y|^2], and the contraction as ONE fmaf chain over
    the 32 slots in the MFMA's order (v_mfma_f32_16x16x4f32 accumulates exactly so:
    tools/mfma_order_probe.py). Slot (s, g) holds feature 16 (s >> 2) + 4 g + (s & 3); slot (6, 3)
    is |emb|^2 x 1, slot (7, 3) is 1 x |y|^2. fmaf is emulated in float64 (exact product, the sum
    rounded to f64 and then to f32: a double rounding can differ from fmaf in 1 ulp, rarely)."""
    ex = np.asarray(ex, np.float32)[:n1, :30]
    ey = np.asarray(ey, np.float32)[:n2, :30]
    C = np.asarray(C, np.float32)

    def fma(a, b, c):
        return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)

    order = [(s, g) for s in range(8) for g in range(4)]
    kid = [16 * (s >> 2) + 4 * g + (s & 3) for s, g in order]
    m2C = (np.float32(-2.0) * C).astype(np.float32)
    emb2 = np.zeros((n1, 32), np.float32)  # -2 emb by feature (30, 31: zero)
    for f in range(30):
        acc = np.zeros(n1, np.float32)
        for k in kid:
            if k < 30:
                acc = fma(np.full(n1, m2C[f, k], np.float32), ex[:, k], acc)
        emb2[:, f] = acc

    def norm(v):  # per lane group g: fmaf chain of the squares over s; groups added in order
        tot = np.zeros(v.shape[0], np.float32)
        for g in range(4):
            p = np.zeros(v.shape[0], np.float32)
            for s in range(8):
                x = v[:, 16 * (s >> 2) + 4 * g + (s & 3)]
                p = fma(x, x, p)
            tot = (tot + p).astype(np.float32)
        return tot

    nA = (np.float32(0.25) * norm(emb2)).astype(np.float32)
    yv = np.zeros((n2, 32), np.float32)
    yv[:, :30] = ey
    nB = norm(yv)
    A = np.zeros((n1, 32), np.float32)
    Bm = np.zeros((n2, 32), np.float32)
    for idx, (s, g) in enumerate(order):
        k = kid[idx]
        A[:, idx] = emb2[:, k] if k < 30 else (nA if k == 30 else 1.0)
        Bm[:, idx] = yv[:, k] if k < 30 else (1.0 if k == 30 else nB)
    acc = np.zeros((n1, n2), np.float32)
    for idx in range(32):
        acc = fma(A[:, idx, None], Bm[None, :, idx], acc)
    return acc


def fd_expected_topk(d, k):
    """torch.cdist's clamp_min(1e-30), then the k smallest rows of every column in ascending
    order, ties to the lower row (the reference's dist.sort order on exact ties: stable), -1 past
    the rows present. Returns (idx [n2, k] int64, clamped values [n2, k] f32)."""
    dc = np.maximum(d, np.float32(1e-30))
    n1, n2 = dc.shape
    order = np.argsort(dc, axis=0, kind="stable")[:k].T
    idx = np.full((n2, k), -1, np.int64)
    val = np.full((n2, k), np.inf, np.float32)
    m = min(k, n1)
    idx[:, :m] = order[:, :m]
    val[:, :m] = np.take_along_axis(dc, order[:, :m].T, axis=0).T
    return idx, val
