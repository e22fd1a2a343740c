"""GPU parity for the model path (H7 spectral diffusion, H8 attention/refinement, H9 fmap
solve, DPFMNet forward + backward) against the torch-CPU oracle restatement, fp32
tolerances stated per test; weights loaded through the reference's state_dict names."""
import numpy as np
import pytest
import torch

from oracle import dpfm_model_oracle as M

pytestmark = pytest.mark.gpu


def _inputs(B, N1, N2, seed=0):
    from dpfm_amd.dataset.synthetic import lbo_operators
    rng = np.random.default_rng(seed)
    out = {}
    for key, n, off in (("shape1", N1, 0), ("shape2", N2, 1)):
        mass, evals, evecs = zip(*[lbo_operators(n, 64, 2 * b + off + seed) for b in range(B)])
        xyz = rng.normal(size=(B, n, 3)).astype(np.float32) * 6 + np.float32(100)
        out[key] = {"xyz": torch.from_numpy(xyz), "mass": torch.from_numpy(np.stack(mass)),
                    "evals": torch.from_numpy(np.stack(evals)), "evecs": torch.from_numpy(np.stack(evecs))}
    return out


def _to(batch, dev):
    return {k: {kk: vv.to(dev) for kk, vv in v.items()} for k, v in batch.items()}


def test_spectral_diffusion_fwd_bwd(device):
    from dpfm_amd import ops
    B, N = 3, 700
    b = _inputs(B, N, N)["shape1"]
    x = torch.randn(B, N, 64, dtype=torch.float32)
    t = torch.rand(64) * 5
    g = torch.randn(B, N, 64)
    # oracle
    xr, tr = x.clone().requires_grad_(), t.clone().requires_grad_()
    spec = torch.matmul(b["evecs"].transpose(-2, -1), xr * b["mass"].unsqueeze(-1))
    yr = torch.matmul(b["evecs"], torch.exp(-b["evals"].unsqueeze(-1) * tr.unsqueeze(0)) * spec)
    (yr * g).sum().backward()
    xd = x.to(device).requires_grad_()
    td = t.to(device).requires_grad_()
    yd = ops.spectral_diffusion(xd, b["mass"].to(device), b["evals"].to(device), b["evecs"].to(device), td)
    (yd * g.to(device)).sum().backward()
    torch.testing.assert_close(yd.detach().cpu(), yr.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(xd.grad.cpu(), xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(td.grad.cpu(), tr.grad, rtol=1e-3, atol=1e-3)


def test_fmap_solve_fwd_bwd(device):
    from dpfm_amd import ops
    from dpfm_amd.dpfm_utils import get_mask_batched
    torch.manual_seed(0)
    B = 4
    A = torch.randn(B, 30, 32, dtype=torch.float64)
    Bm = torch.randn(B, 30, 32, dtype=torch.float64)
    ex = torch.sort(torch.rand(B, 30) * 2, dim=1).values
    ey = torch.sort(torch.rand(B, 30) * 2, dim=1).values
    D = get_mask_batched(ex, ey, 0.5).to(torch.float64)
    G = torch.randn(B, 30, 30, dtype=torch.float64)
    # fp64 ground truth of modeling/dpfm.py:185-193
    Ar = A.clone().requires_grad_()
    Br = Bm.clone().requires_grad_()
    AAt, BAt = Ar @ Ar.transpose(1, 2), Br @ Ar.transpose(1, 2)
    rows = [torch.linalg.solve(AAt + 100.0 * torch.diag_embed(D[:, i, :]), BAt[:, i, :, None]).transpose(1, 2)
            for i in range(30)]
    Cr = torch.cat(rows, 1)
    (Cr * G).sum().backward()
    Ad = A.float().to(device).requires_grad_()
    Bd = Bm.float().to(device).requires_grad_()
    AAtd, BAtd = Ad @ Ad.transpose(1, 2), Bd @ Ad.transpose(1, 2)
    Cd = ops.fmap_solve(AAtd, BAtd, D.float().to(device), 100.0)
    (Cd * G.float().to(device)).sum().backward()
    scale = Cr.abs().max()
    torch.testing.assert_close(Cd.detach().cpu().double(), Cr.detach(), rtol=1e-3, atol=1e-4 * float(scale))
    torch.testing.assert_close(Ad.grad.cpu().double(), Ar.grad, rtol=1e-3, atol=1e-3 * float(Ar.grad.abs().max()))
    torch.testing.assert_close(Bd.grad.cpu().double(), Br.grad, rtol=1e-3, atol=1e-3 * float(Br.grad.abs().max()))


@pytest.mark.parametrize("shape,channels_first", [((32768, 128, 64), False), ((1000, 3, 64), False),
                                                  ((4, 7, 32, 1), False), ((3, 32, 300, 64), True),
                                                  ((2, 64, 1024, 32), True), ((0, 8, 8), False)])
def test_linear_wgrad(device, shape, channels_first):
    """pk_linear_wgrad vs fp64: |err| <= 1e-5 * sum_r |dy||x| (the fp32 summation bound)."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(sum(shape))
    if channels_first:
        Bn, I, N, O = shape
        x = torch.randn(Bn, I, N, generator=g)
        dy = torch.randn(Bn, O, N, generator=g)
        exp_w = torch.einsum("bon,bin->oi", dy.double(), x.double())
        bound = torch.einsum("bon,bin->oi", dy.double().abs(), x.double().abs())
        exp_b, bnd_b = dy.double().sum((0, 2)), dy.double().abs().sum((0, 2))
    else:
        *lead, I, O = shape
        x = torch.randn(*lead, I, generator=g)
        dy = torch.randn(*lead, O, generator=g)
        x2, d2 = x.reshape(-1, I).double(), dy.reshape(-1, O).double()
        exp_w, bound = d2.t() @ x2, d2.abs().t() @ x2.abs()
        exp_b, bnd_b = d2.sum(0), d2.abs().sum(0)
    dw, db = ops.linear_wgrad(x.to(device), dy.to(device), channels_first=channels_first)
    assert (dw.cpu().double() - exp_w).abs().le(1e-5 * bound + 1e-30).all()
    assert (db.cpu().double() - exp_b).abs().le(1e-5 * bnd_b + 1e-30).all()


def test_linear_wgrad_grouped(device):
    """pk_linear_wgrad_grouped (every layer of a backward in two launches) vs fp64 per call:
    both layouts, a shared layer fed by two calls (accumulate), an empty call, a layer
    whose only call is empty (zero gradient), thin operands and ragged last tiles on the LDS-DMA
    pipeline, and > 32 calls (several table chunks)."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(11)
    specs = [  # (lead shape, I, O, channels_first, shared-with index or None)
        ((64, 1024), 128, 64, False, None), ((64, 1024), 64, 64, False, None), ((3, 700), 3, 64, False, None),
        ((32, 1024), 32, 32, True, None), ((32, 1024), 64, 32, True, None), ((32, 1024), 32, 32, True, 3),
        ((0,), 16, 8, False, None), ((5, 33), 64, 32, False, None), ((2, 1024), 64, 64, True, 1 << 30),
        ((3, 5002), 64, 32, True, None), ((2, 300), 64, 32, True, 9),  # ragged items (N % 16 != 0)
        ((65536,), 3, 64, False, None), ((4, 1001), 32, 1, False, None),  # thin operands (3 -> 64, 32 -> 1)
        ((2, 32768), 128, 64, False, None),
    ]
    specs = specs + [((7, 48), 32, 32, False, None)] * 30
    calls, exp = [], {}
    for k, (lead, I, O, cf, shared) in enumerate(specs):
        if cf:
            Bn, N = lead
            x, dy = torch.randn(Bn, I, N, generator=g), torch.randn(Bn, O, N, generator=g)
            ew, eb = torch.einsum("bon,bin->oi", dy.double(), x.double()), dy.double().sum((0, 2))
            bw = torch.einsum("bon,bin->oi", dy.double().abs(), x.double().abs())
        else:
            x, dy = torch.randn(*lead, I, generator=g), torch.randn(*lead, O, generator=g)
            x2, d2 = x.reshape(-1, I).double(), dy.reshape(-1, O).double()
            ew, eb, bw = d2.t() @ x2, d2.sum(0), d2.abs().t() @ x2.abs()
        if shared is not None and shared < len(calls):
            dw, db = calls[shared][3], calls[shared][4]
            e = exp[shared]
            exp[shared] = (e[0] + ew, e[1] + eb, e[2] + bw)
            calls.append((x.to(device), dy.to(device), cf, dw, db, True))
        else:
            dw = torch.full((O, I), float("nan"), device=device)
            db = torch.full((O,), float("nan"), device=device)
            exp[k] = (ew, eb, bw)
            calls.append((x.to(device), dy.to(device), cf, dw, db, False))
    ops.linear_wgrad_grouped(calls)
    torch.cuda.synchronize()
    for k, (ew, eb, bw) in exp.items():
        dw, db = calls[k][3].cpu().double(), calls[k][4].cpu().double()
        assert (dw - ew).abs().le(1e-5 * bw + 1e-30).all(), k
        assert (db - eb).abs().le(1e-5 * bw.max() + 1e-30).all(), k


@pytest.mark.parametrize("N,M", [(300, 200), (1024, 1024), (64, 1), (17, 130), (77, 600), (5, 513), (130, 257)])
def test_attention_fwd_bwd(device, N, M):
    """H8 fused attention vs modeling/dpfm.py:29-37 evaluated in fp64 (truth) and fp32:
    out and dq/dk/dv within 3x the fp32 reference's own error + 1e-6 of scale."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(N * 7 + M)
    B, D, H = 3, 16, 2
    q = torch.randn(B, D, H, N, generator=g) * 2
    k = torch.randn(B, D, H, M, generator=g) * 2
    v = torch.randn(B, D, H, M, generator=g)
    go = torch.randn(B, D, H, N, generator=g)

    def ref(q, k, v):
        scores = torch.einsum("bdhn,bdhm->bhnm", q, k) / D ** 0.5
        return torch.einsum("bhnm,bdhm->bdhn", torch.nn.functional.softmax(scores, dim=-1), v)

    res = []
    for dt, dev in ((torch.float64, "cpu"), (torch.float32, "cpu"), (torch.float32, device)):
        ins = [x.detach().clone().to(device=dev, dtype=dt).requires_grad_() for x in (q, k, v)]
        out = (ops.attention if dev == device else ref)(*ins)
        (out * go.to(device=dev, dtype=dt)).sum().backward()
        res.append([t.detach().cpu().double() for t in (out, *(x.grad for x in ins))])
    scale = max(t.abs().max().item() for t in res[0])  # M = 1: dk vanishes exactly in truth
    for name, t, r, d in zip(["out", "dq", "dk", "dv"], *res):
        e_ref, e_mine = (r - t).abs().max().item(), (d - t).abs().max().item()
        assert e_mine <= 3 * e_ref + 1e-6 * (1 + scale), (name, e_mine, e_ref)


def test_attention_bwd_deterministic_any_scratch(device):
    """The one-pass backward's dQ partials (one per 256-key block, slot 0 = dq) are added in
    slot order: two calls agree bit for bit, whatever the work buffer held before."""
    import ctypes
    from dpfm_amd import _lib, ops
    g = torch.Generator().manual_seed(11)
    B, D, H, N, M = 2, 16, 2, 333, 1100
    q, k, v, go = (torch.randn(B, D, H, n, generator=g).to(device) for n in (N, M, M, N))
    out = torch.empty_like(q)
    lse = torch.empty((B, H, N, 2), device=device)
    P = _lib.ptr
    _lib.call("pk_attention_fwd", P(q), P(k), P(v), B, D, H, N, M, 0, 0, P(out), P(lse), _lib.stream(device))
    res = []
    for fill in (0.0, float("nan"), 1e30):
        work = ops.attention_bwd_work(B, D, H, N, M, device)
        assert work is not None and work.numel() == 4 * B * D * H * N  # 5 key blocks: 4 extra slots
        work.fill_(fill)
        dq, dk, dv = torch.full_like(q, fill), torch.empty_like(k), torch.empty_like(v)
        _lib.call("pk_attention_bwd", P(q), P(k), P(v), P(out), P(go), P(lse), B, D, H, N, M, 0, 0, P(work),
                  P(dq), P(dk), P(dv), 0, 0, _lib.stream(device))
        res.append((dq.cpu(), dk.cpu(), dv.cpu()))
    for r in res[1:]:
        for a, b in zip(res[0], r):
            assert torch.equal(a, b)
    assert ops.attention_bwd_work(B, D, H, N, 256, device) is None  # one key block: no scratch


@pytest.mark.parametrize("N1,N2", [(256, 256), (300, 200)])
def test_dpfmnet_matches_oracle(device, N1, N2):
    """Forward outputs and parameter gradients vs the oracle evaluated in fp64 (the truth).
    Yardstick: the same oracle evaluated in fp32, on the CPU (the reference's own path) and
    with torch on the GPU; the HIP path must be within 3x the larger of their errors.
    Gradients are compared as Frobenius norms per parameter (max-abs errors of independent
    fp32 evaluations fluctuate by several x), with an absolute floor of 1e-6 x the global
    gradient norm for the parameters whose true gradient vanishes by invariance (biases in
    front of InstanceNorm / the softmax's key bias)."""
    from dpfm_amd.models.dpfm import DPFMNet
    torch.manual_seed(3)
    ref = M.DPFMNet()
    with torch.no_grad():  # exercise the in-place clamp with negative diffusion times
        ref.feature_extractor.block_0.diffusion.diffusion_time.uniform_(-0.001, 12)
        ref.feature_extractor.block_1.diffusion.diffusion_time.uniform_(-0.001, 12)
    truth = M.DPFMNet().double()
    truth.load_state_dict(ref.state_dict())
    gref = M.DPFMNet().to(device)
    gref.load_state_dict(ref.state_dict())
    mine = DPFMNet().to(device)
    mine.load_state_dict(ref.state_dict(), strict=True)
    batch = _inputs(2, N1, N2, seed=5)
    batch64 = {k: {kk: vv.double() for kk, vv in v.items()} for k, v in batch.items()}
    runs = [(truth, batch64), (ref, batch), (gref, _to(batch, device)), (mine, _to(batch, device))]

    outs = [m(b) for m, b in runs]
    for n, t, r, g, d in zip(["C", "o12", "o21", "f1", "f2"], *(o[:5] for o in outs)):
        t = t.detach()
        e = [(x.detach().cpu().double() - t).abs().max().item() for x in (r, g, d)]
        assert e[2] <= 3 * max(e[0], e[1]) + 1e-6 * (1 + t.abs().max().item()), (n, e)

    def check(loss_fn):
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
            assert e[2] <= 3 * max(e[0], e[1]) + floor, (name, e, floor)

    check(lambda o: o[1].sum() + o[2].sum() + o[3].square().sum() + o[4].square().sum())  # overlap + features
    check(lambda o: o[0].sum())                                                          # through the fmap solve


@pytest.mark.parametrize("shape,channels_first,transw", [((65536, 128, 64), False, False), ((1000, 3, 64), False, False),
                                                          ((4, 7, 32, 1), False, False), ((3, 32, 300, 64), True, False),
                                                          ((2, 64, 1024, 32), True, False), ((4096, 64, 128), False, True),
                                                          ((2, 64, 512, 32), True, True), ((0, 8, 8), False, False),
                                                          ((32, 64, 1024, 64), True, False), ((64, 32, 2048, 128), True, False),
                                                          ((32, 128, 1024, 64), True, True), ((3, 16, 48, 5), True, False),
                                                          ((5000, 32, 1), False, False), ((777, 16, 100), False, True),
                                                          ((32, 32, 1024, 1), True, False), ((32, 1, 1024, 32), True, True),
                                                          ((3, 2, 100, 7), True, False), ((10, 33, 3), False, True),
                                                          ((2, 40, 64, 3), True, True), ((65536, 3, 64), False, False),
                                                          # ragged channels-first items (N % 16 != 0: tiles end per item)
                                                          ((2, 64, 5002, 32), True, True), ((3, 128, 203, 64), True, False),
                                                          ((2, 16, 7, 20), True, False)])
def test_linear_fwd(device, shape, channels_first, transw):
    """pk_linear_fwd (per-point layer forward, bias fused; transw = the input gradient dy W)
    vs fp64: |err| <= 1e-5 * sum_k |x||w| + 1e-6 |b|."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(sum(shape) + 7 * transw)
    if channels_first:
        Bn, I, N, O = shape
        x = torch.randn(Bn, I, N, generator=g)
    else:
        *lead, I, O = shape
        x = torch.randn(*lead, I, generator=g)
    w = torch.randn(O, I, generator=g) * 0.2
    b = None if transw else torch.randn(O, generator=g)
    w_arg = w.t().contiguous() if transw else w  # transw: the kernel reads W^T of a [Cin, Cout] tensor
    y = ops.linear_fwd(x.to(device), w_arg.to(device), None if b is None else b.to(device),
                       channels_first=channels_first, transw=transw).cpu().double()
    xd, wd = x.double(), w.double()
    if channels_first:
        exp = torch.einsum("oi,bin->bon", wd, xd)
        bound = torch.einsum("oi,bin->bon", wd.abs(), xd.abs())
        if b is not None:
            exp = exp + b.double()[None, :, None]
    else:
        exp, bound = xd @ wd.t(), xd.abs() @ wd.abs().t()
        if b is not None:
            exp = exp + b.double()
    assert y.shape == exp.shape
    assert (y - exp).abs().le(1e-5 * bound + 1e-6 * (0 if b is None else b.abs().max().item()) + 1e-30).all()


@pytest.mark.parametrize("R,I,O,epi", [(65536, 128, 64, "relu"), (65536, 64, 64, "add"), (65536, 64, 128, "split_add"),
                                        (65536, 64, 64, "mask"), (40000, 128, 32, "mask_add"), (4099, 32, 128, "split"),
                                        (17, 64, 64, "mask_add"), (300000, 64, 64, "relu"), (65536, 64, 32, "plain")])
def test_linear_ex_rows_epilogues(device, R, I, O, epi):
    """pk_linear_ex on the rows layout (the LDS-DMA pipeline for Cin, Cout in {32, 64, 128}) with the
    step's epilogues vs fp64: ReLU; the ReLU-backward mask; a residual added to the first add_cols
    outputs from a wider row-strided buffer; outputs >= split to a second strided tensor; R with a
    partial last tile and many tiles per wave. Bound |err| <= 1e-5 sum_k |x||w| (+ |b|, |add|
    rounding)."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(R + I + O)
    ldx = I + 16
    xs = torch.randn(R, ldx, generator=g)
    x = xs[:, :I]
    w = torch.randn(O, I, generator=g) * 0.2
    b = torch.randn(O, generator=g)
    dev = device
    xd, wd = x.double(), w.double()
    exp = xd @ wd.t() + b.double()
    bound = xd.abs() @ wd.abs().t() * 1e-5 + 1e-6 * b.abs().max().item()
    relu = epi in ("relu",)
    if relu:
        exp = exp.clamp_min(0)
    mask = None
    if "mask" in epi:
        mask = torch.randn(R, O, generator=g)
        exp = torch.where(mask.double() <= 0, torch.zeros_like(exp), exp)
    add = None
    add_cols = 0
    lda = 0
    if "add" in epi:
        add_cols = O // 2
        lda = O + 8
        add = torch.randn(R, lda, generator=g)
        exp[:, :add_cols] += add[:, :add_cols].double()
        bound[:, :add_cols] += 1e-6 * add[:, :add_cols].abs().double()
    split = O // 2 if "split" in epi else 0
    ldy = O + 4 if not split else split + 4
    y = torch.full((R, ldy), float("nan"), device=dev)
    y2 = torch.full((R, O - split + 12), float("nan"), device=dev) if split else None
    xg = xs.to(dev)
    ops.linear_ex(xg, w.to(dev), b.to(dev), 0, R, 0, I, O, y, ldx=ldx, ldy=ldy, relu=relu,
                  mask=None if mask is None else mask.to(dev), add=None if add is None else add.to(dev), lda=lda,
                  add_cols=add_cols, y2=y2, split=split, ldy2=0 if y2 is None else y2.shape[1])
    got = y.cpu().double()
    if split:
        full = torch.cat([got[:, :split], y2.cpu().double()[:, :O - split]], 1)
        assert torch.isnan(got[:, split:]).all() and torch.isnan(y2.cpu()[:, O - split:]).all()
    else:
        full = got[:, :O]
        assert torch.isnan(got[:, O:]).all()  # nothing written past the row's outputs
    assert (full - exp).abs().le(bound + 1e-30).all(), float(((full - exp).abs() - bound).max())


def test_dpfm_loss_matches_oracle(device):
    """H15 DPFMLoss (Frobenius + fused NCE kernel pk_nce_loss + weighted BCE, batched over
    crops) vs the reference loss restated in fp64 on the CPU (utils/loss.py:8-99), on the
    same NCE pair draw: loss within 1e-4 relative, every input gradient within 1e-4 of its
    scale. Crops with more pairs than 512 (draw without replacement), fewer, exactly 512,
    and repeated CAD / crop indices (one point in several pairs)."""
    from dpfm_amd import ops
    from dpfm_amd.utils.loss import DPFMLoss
    g = torch.Generator().manual_seed(5)
    B, N1, N2 = 4, 700, 600
    counts = [1500, 300, 512, 2000]
    cap = max(counts)
    pairs = torch.zeros((B, cap, 2), dtype=torch.int64)
    for b, c in enumerate(counts):
        flat = torch.randperm(N1 * N2, generator=g)[:c]
        pairs[b, :c, 0] = flat // N2
        pairs[b, :c, 1] = flat % N2
        if b == 3:  # many pairs on a few CAD points
            pairs[b, :c, 0] = pairs[b, :c, 0] % 37
    f1 = torch.randn(B, N1, 32, generator=g)
    f2 = torch.randn(B, N2, 32, generator=g)
    C = torch.randn(B, 30, 30, generator=g)
    C_gt = torch.randn(B, 30, 30, generator=g)
    # crops 0-1 below FrobeniusLoss's clamp (sum ~ 225 < 1000: gradient flows), 2-3 above it
    C_gt[:2] = C[:2] + 0.5 * torch.randn(2, 30, 30, generator=g)
    o12 = torch.rand(B, N1, generator=g) * 0.98 + 0.01
    o21 = torch.rand(B, N2, generator=g) * 0.98 + 0.01
    g12 = (torch.rand(B, N1, generator=g) < 0.4).to(torch.int8)
    g21 = (torch.rand(B, N2, generator=g) < 0.6).to(torch.int8)
    npairs = torch.tensor(counts, dtype=torch.int64)
    ctr = torch.zeros(1, dtype=torch.int64, device=device)
    rows, valid = ops.nce_select(npairs.to(device), cap, 512, 9, ctr)
    sel = [rows[b][valid[b]].cpu() for b in range(B)]
    assert [len(s) for s in sel] == [512, 300, 512, 512]
    # device (fp32)
    dv = [t.to(device).requires_grad_(True) for t in (C, f1, f2, o12, o21)]
    crit = DPFMLoss(w_fmap=1, w_acc=1, w_nce=1, nce_t=0.07, nce_num_pairs=512)
    loss, _ = crit.forward_batched(dv[0], C_gt.to(device), pairs.to(device), npairs.to(device), dv[1], dv[2],
                                   dv[3], dv[4], g12.to(device), g21.to(device), selection=(rows, valid))
    loss.backward()
    # oracle (fp64, CPU)
    rv = [t.double().requires_grad_(True) for t in (C, f1, f2, o12, o21)]
    plist = [pairs[b, :counts[b]] for b in range(B)]
    ref = M.dpfm_loss(rv[0], C_gt.double(), plist, sel, rv[1], rv[2], rv[3], rv[4], g12, g21)
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 1e-4 * abs(float(ref)), (float(loss), float(ref))
    assert rv[0].grad[:2].abs().max() > 0 and rv[0].grad[2:].abs().max() == 0  # both clamp regimes covered
    for name, a, r in zip(("C", "f1", "f2", "o12", "o21"), dv, rv):
        ga, gr = a.grad.cpu().double(), r.grad
        scale = float(gr.abs().max())
        assert (ga - gr).abs().max().item() <= 1e-4 * scale + 1e-9, (name, (ga - gr).abs().max().item(), scale)


def test_nce_loss_edge_cases(device):
    """pk_nce_loss: a crop without pairs has loss 0 and zero gradients; no-grad calls skip
    the gradient pass and give the same loss."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(8)
    B, N = 3, 64
    counts = torch.tensor([0, 5, 64], dtype=torch.int64)
    pairs = torch.zeros((B, 64, 2), dtype=torch.int64)
    for b in range(B):
        pairs[b, :, 0] = torch.randperm(N, generator=g)
        pairs[b, :, 1] = torch.randperm(N, generator=g)
    ctr = torch.zeros(1, dtype=torch.int64, device=device)
    rows, valid = ops.nce_select(counts.to(device), 64, 512, 1, ctr)
    f1 = torch.randn(B, N, 32, generator=g).to(device).requires_grad_(True)
    f2 = torch.randn(B, N, 32, generator=g).to(device).requires_grad_(True)
    loss = ops.nce_loss(f1, f2, pairs.to(device), rows, valid, 0.07)
    loss.sum().backward()
    assert float(loss[0]) == 0.0 and float(f1.grad[0].abs().max()) == 0.0 and float(f2.grad[0].abs().max()) == 0.0
    with torch.no_grad():
        l2 = ops.nce_loss(f1, f2, pairs.to(device), rows, valid, 0.07)
    assert torch.equal(loss.detach(), l2)
    # channels-first storage (the refinement net's ref_feat layout) is read in place
    cf = lambda t: t.detach().transpose(1, 2).contiguous().transpose(1, 2).requires_grad_(True)  # noqa: E731
    f1c, f2c = cf(f1), cf(f2)
    assert not f1c.is_contiguous()
    l3 = ops.nce_loss(f1c, f2c, pairs.to(device), rows, valid, 0.07)
    l3.sum().backward()
    assert torch.equal(loss.detach(), l3.detach())
    assert torch.equal(f1c.grad, f1.grad) and torch.equal(f2c.grad, f2.grad)
    for b in (1, 2):
        s = rows[b][valid[b]].cpu()
        r = M.nce_loss(f1[b].detach().cpu().double(), f2[b].detach().cpu().double(), pairs[b, :int(counts[b])], s)
        assert abs(float(loss[b]) - float(r)) <= 1e-4 * abs(float(r))


def test_nce_gradients_deterministic(device):
    """pk_nce_loss sums the slot gradient rows of a point in ascending slot order (no float
    atomics): repeated calls, and rows vs channels-first storage, give bit-identical gradients,
    also when most slots share a handful of points; the sums match the fp64 oracle."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(12)
    B, N1, N2, cap = 3, 300, 400, 900
    pairs = torch.stack([torch.randint(0, N1, (B, cap), generator=g), torch.randint(0, N2, (B, cap), generator=g)], -1)
    pairs[1, :, 0] %= 3      # every CAD slot on 3 points
    pairs[2, :, 1] %= 7      # every crop slot on 7 points
    counts = torch.tensor([cap, cap, 200], dtype=torch.int64)
    ctr = torch.zeros(1, dtype=torch.int64, device=device)
    rows, valid = ops.nce_select(counts.to(device), cap, 512, 3, ctr)
    f1 = torch.randn(B, N1, 32, generator=g).to(device)
    f2 = torch.randn(B, N2, 32, generator=g).to(device)
    pd = pairs.to(device)
    outs = [ops._nce_raw(f1, f2, pd, rows, valid.view(torch.uint8), 0.07, True) for _ in range(3)]
    f1c, f2c = f1.transpose(1, 2).contiguous().transpose(1, 2), f2.transpose(1, 2).contiguous().transpose(1, 2)
    outs.append(ops._nce_raw(f1c, f2c, pd, rows, valid.view(torch.uint8), 0.07, True))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)
    for b in range(B):
        s = rows[b][valid[b]].cpu()
        r1 = f1[b].detach().cpu().double().requires_grad_(True)
        r2 = f2[b].detach().cpu().double().requires_grad_(True)
        ref = M.nce_loss(r1, r2, pairs[b, :int(counts[b])], s)
        ref.backward()
        for ga, gr in ((outs[0][1][b], r1.grad), (outs[0][2][b], r2.grad)):
            scale = float(gr.abs().max())
            assert (ga.cpu().double() - gr).abs().max().item() <= 1e-4 * scale + 1e-9


@pytest.mark.parametrize("B,C,N", [(4, 64, 1024), (3, 64, 300), (2, 8, 4096), (2, 16, 2048)])
def test_instnorm_relu_fwd_bwd(device, B, C, N):
    """Fused InstanceNorm1d(C) + ReLU (modeling/dpfm.py:16-26) vs torch in fp64: output and
    input gradient within 1e-5 of scale; register-tile (N <= 2048) and streaming paths."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(B * C + N)
    x = torch.randn(B, C, N, generator=g) * 3 + 1
    dy = torch.randn(B, C, N, generator=g)
    xr = x.double().requires_grad_(True)
    yr = torch.relu(torch.nn.functional.instance_norm(xr, eps=1e-5))
    yr.backward(dy.double())
    xd = x.to(device).requires_grad_(True)
    yd = ops.instnorm_relu(xd, 1e-5)
    yd.backward(dy.to(device))
    assert (yd.detach().cpu().double() - yr.detach()).abs().max().item() <= 1e-5 * yr.abs().max().item()
    assert (xd.grad.cpu().double() - xr.grad).abs().max().item() <= 1e-5 * xr.grad.abs().max().item()


@pytest.mark.parametrize("cf", [False, True])
def test_l2_normalize_fwd_bwd(device, cf):
    """Fused F.normalize(x, p=2, dim=-1) (overlap head, modeling/dpfm.py:140-141) vs torch in
    fp64, rows and channels-first storage, including an all-zero point (the eps clamp)."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(3 + cf)
    x = torch.randn(3, 257, 32, generator=g)
    x[1, 7] = 0.0
    dy = torch.randn(3, 257, 32, generator=g)
    xr = x.double().requires_grad_(True)
    yr = torch.nn.functional.normalize(xr, p=2, dim=-1)
    yr.backward(dy.double())
    xd = x.to(device)
    if cf:
        xd = xd.transpose(1, 2).contiguous().transpose(1, 2)
    xd.requires_grad_(True)
    yd = ops.l2_normalize(xd)
    assert yd.stride() == xd.stride()
    yd.backward(dy.to(device))
    assert (yd.detach().cpu().double() - yr.detach()).abs().max().item() <= 1e-6
    scale = xr.grad.abs().max().item()
    assert (xd.grad.cpu().double() - xr.grad).abs().max().item() <= 1e-5 * scale


def test_block_mlp_fused_matches_layers(device):
    """H7 DiffusionNet block MLP: the fused forward (pk_mlp3_fwd: cat + 3 layers + ReLUs +
    residual in one launch) equals the per-layer path bit for bit (same MFMA accumulation
    order); its backward's input and parameter gradients agree within 1e-5 of scale."""
    from dpfm_amd.diffusion_net import DiffusionNetBlock
    torch.manual_seed(2)
    blk = DiffusionNetBlock(C_width=64, mlp_hidden_dims=[64, 64], dropout=False).to(device)
    blk.fused_mlp = True  # opt-in path (DiffusionNetBlock.fused_mlp)
    assert blk._fusable(torch.zeros(1, device=device))
    g = torch.Generator().manual_seed(9)
    B, N = 4, 700
    x = torch.randn(B, N, 64, generator=g).to(device)
    mass = torch.rand(B, N, generator=g).to(device) * 1e-3
    evals = torch.sort(torch.rand(B, 64, generator=g) * 2, dim=1)[0].to(device)
    evecs = torch.randn(B, N, 64, generator=g).to(device) * 0.1
    dy = torch.randn(B, N, 64, generator=g).to(device)
    outs = {}
    for fused in (True, False):
        blk.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        if not fused:
            blk._fusable = lambda _x: False
        y = blk(xi, mass, None, evals, evecs, None, None)
        if not fused:
            del blk._fusable
        y.backward(dy)
        outs[fused] = (y.detach(), xi.grad.detach(), [p.grad.detach().clone() for p in blk.parameters()])
    assert torch.equal(outs[True][0], outs[False][0])
    for a, b in [(outs[True][1], outs[False][1])] + list(zip(outs[True][2], outs[False][2])):
        assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item() + 1e-12


def test_resolvent_mask_matches_get_mask(device):
    """pk_resolvent_mask (all crops, one launch) vs upstream get_mask per crop (restated in
    dpfm_utils.get_mask) in fp64, on sliced [:, :30] views of [B, 64] eigenvalues."""
    from dpfm_amd import ops
    from dpfm_amd.dpfm_utils import get_mask
    g = torch.Generator().manual_seed(12)
    B = 5
    e1 = torch.sort(torch.rand(B, 64, generator=g) * 3, dim=1)[0]
    e2 = torch.sort(torch.rand(B, 64, generator=g) * 5, dim=1)[0]
    e1[:, 0] = 0.0
    D = ops.resolvent_mask(e1.to(device)[:, :30], e2.to(device)[:, :30], 0.5).cpu().double()
    for b in range(B):
        ref = get_mask(e1[b, :30].double(), e2[b, :30].double(), 0.5)
        assert (D[b] - ref).abs().max().item() <= 1e-6 * ref.abs().max().item() + 1e-12


def test_relu_backward_folded_into_dgrad(device, monkeypatch):
    """The fused ReLU's backward folded into the next layer's input-gradient epilogue
    (pk_linear_fwd mask) gives the same DiffusionNet input and parameter gradients, bit for
    bit, as applying aten threshold_backward separately."""
    from dpfm_amd import diffusion_net as DN
    from dpfm_amd import layers
    monkeypatch.setattr(DN, "FUSED_ENCODER", False)  # the per-module path is the one that folds
    from dpfm_amd.diffusion_net import DiffusionNet
    torch.manual_seed(6)
    net = DiffusionNet(C_in=3, C_out=32, C_width=64, N_block=2, dropout=False,
                       with_gradient_features=False).to(device)
    b = _to(_inputs(2, 512, 512, seed=3), device)["shape1"]
    x = ((b["xyz"] - 110) / 50).requires_grad_(True)
    g = torch.Generator().manual_seed(1)
    dy = torch.randn(2, 512, 32, generator=g).to(device)
    res = {}
    for fold in (True, False):
        layers.FOLD_RELU = fold
        net.zero_grad(set_to_none=True)
        x.grad = None
        net(x, b["mass"], evals=b["evals"], evecs=b["evecs"]).backward(dy)
        res[fold] = [x.grad.clone()] + [p.grad.clone() for p in net.parameters()]
    layers.FOLD_RELU = True
    for a, c in zip(res[True], res[False]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("B,N", [(3, 256), (2, 333)])
def test_fused_encoder_matches_module_path(device, B, N, monkeypatch):
    """The DiffusionNet encoder as one autograd node (_EncoderFn: concatenation-free blocks,
    residual adds and split input gradients in the layer epilogues, diffusion backward
    accumulated in place) against the per-module path (FUSED_ENCODER = False) on the same
    weights: forward bit-identical (same kernels and per-element arithmetic), gradients of
    every parameter within 2e-5 of their scale (only the order of the residual / diffusion
    gradient sums differs)."""
    from dpfm_amd import diffusion_net as DN
    from dpfm_amd.models.dpfm import DPFMNet
    torch.manual_seed(11)
    net = DPFMNet().feature_extractor.to(device)
    b = _to(_inputs(B, N, N, seed=3), device)["shape1"]
    x = ((b["xyz"] - 110) / 50).contiguous()
    g = torch.randn(B, N, 32, device=device)
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setattr(DN, "FUSED_ENCODER", mode == "1")
        net.zero_grad(set_to_none=True)
        for blk in net.blocks:  # above the clamp: both paths see the same diffusion times
            blk.diffusion.diffusion_time.data.copy_(torch.linspace(0.01, 2.0, 64, device=device))
        y = net(x, b["mass"], evals=b["evals"], evecs=b["evecs"])
        (y * g).sum().backward()
        res[mode] = (y.detach().clone(), {k: p.grad.detach().clone() for k, p in net.named_parameters()})
    assert torch.equal(res["1"][0], res["0"][0])
    for k, g0 in res["0"][1].items():
        g1 = res["1"][1][k]
        scale = float(g0.abs().max()) + 1e-30
        assert (g1 - g0).abs().max().item() <= 2e-5 * scale, (k, (g1 - g0).abs().max().item(), scale)


@pytest.mark.parametrize("cf,N1,N2", [(True, 1024, 1024), (True, 300, 203), (False, 257, 130)])
def test_fused_overlap_head_matches_layer_path(device, cf, N1, N2, monkeypatch):
    """OverlapPredictorNet (modeling/dpfm.py:125-145) for both shapes in one launch per direction
    (ops.overlap_head) against the per-layer path (l2 normalize, 32 -> 32 MFMA layer, thin
    32 -> 1 sigmoid layer) on the same weights and inputs, channels-first and rows storage, ragged
    N: scores, the NCE rows copies and the feature gradients (with an NCE-like rows gradient
    added) bit-identical — same operations in the same order; weight gradients within 1e-5 of
    their scale (the weight-gradient reduction reads rows instead of channels-first operands)."""
    from dpfm_amd.modeling import dpfm as mdp
    torch.manual_seed(5)
    head = mdp.OverlapPredictorNet(32).to(device)
    B = 3
    g = torch.Generator().manual_seed(9)

    def feats(N):
        t = torch.randn(B, 32, N, generator=g) if cf else torch.randn(B, N, 32, generator=g)
        if cf:  # a few zero points (the clamped norm branch)
            t[0, :, :3] = 0.0
        else:
            t[0, :3, :] = 0.0
        t = t.to(device)
        return t.transpose(1, 2) if cf else t

    fx0, fy0 = feats(N1), feats(N2)
    ws = (torch.randn(B, N1, generator=g).to(device), torch.randn(B, N2, generator=g).to(device))
    wr = (torch.randn(B, N1, 32, generator=g).to(device), torch.randn(B, N2, 32, generator=g).to(device))
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(mdp, "FUSED_OVERLAP_HEAD", fused)
        head.zero_grad(set_to_none=True)
        fx, fy = fx0.detach().clone().requires_grad_(True), fy0.detach().clone().requires_grad_(True)
        sx, sy = head(fx, fy)
        rx, ry = fx._pk_nrows, fy._pk_nrows
        loss = (sx * ws[0]).sum() + (sy * ws[1]).sum() + (rx * wr[0]).sum() + (ry * wr[1]).sum()
        loss.backward()
        res[fused] = ([t.detach().clone() for t in (sx, sy, rx, ry, fx.grad, fy.grad)],
                      {k: p.grad.detach().clone() for k, p in head.named_parameters()})
    for a, b in zip(res[True][0], res[False][0]):
        assert a.shape == b.shape and torch.equal(a, b), (a - b).abs().max().item()
    for k, g0 in res[False][1].items():
        g1 = res[True][1][k]
        scale = float(g0.abs().max()) + 1e-30
        assert (g1 - g0).abs().max().item() <= 1e-5 * scale, (k, (g1 - g0).abs().max().item(), scale)


def test_nce_on_prenormalized_rows_matches_raw(device):
    """The NCE term fed the overlap head's F.normalize'd rows copy (ops.l2_normalize_two,
    pk_nce_loss prenorm = 1, its gradient joining the l2-normalize backward) against the term
    normalizing the raw channels-first features itself: same loss and feature gradients
    within f32 rounding of the two norm evaluations (1e-5 of scale)."""
    from dpfm_amd import ops
    from dpfm_amd.utils.loss import DPFMLoss
    g = torch.Generator().manual_seed(12)
    B, N1, N2 = 3, 300, 260
    counts = [700, 40, 512]
    cap = max(counts)
    pairs = torch.zeros((B, cap, 2), dtype=torch.int64)
    for b, c in enumerate(counts):
        flat = torch.randperm(N1 * N2, generator=g)[:c]
        pairs[b, :c, 0], pairs[b, :c, 1] = flat // N2, flat % N2
    f1 = torch.randn(B, 32, N1, generator=g).to(device).transpose(1, 2)  # channels-first storage
    f2 = torch.randn(B, 32, N2, generator=g).to(device).transpose(1, 2)
    C = torch.randn(B, 30, 30, generator=g).to(device)
    C_gt = torch.randn(B, 30, 30, generator=g).to(device)
    o12 = (torch.rand(B, N1, generator=g) * 0.9 + 0.05).to(device)
    o21 = (torch.rand(B, N2, generator=g) * 0.9 + 0.05).to(device)
    t12 = (torch.rand(B, N1, generator=g) < 0.5).to(torch.int8).to(device)
    t21 = (torch.rand(B, N2, generator=g) < 0.5).to(torch.int8).to(device)
    npairs = torch.tensor(counts, device=device)
    ctr = torch.zeros(1, dtype=torch.int64, device=device)
    rows, valid = ops.nce_select(npairs, cap, 512, 3, ctr)
    crit = DPFMLoss(w_fmap=1, w_acc=1, w_nce=1, nce_t=0.07, nce_num_pairs=512)
    res = []
    for pre in (False, True):
        a1, a2 = f1.detach().clone().requires_grad_(True), f2.detach().clone().requires_grad_(True)
        if pre:
            _, a1._pk_nrows = ops.l2_normalize_two(a1)
            _, a2._pk_nrows = ops.l2_normalize_two(a2)
        loss, _ = crit.forward_batched(C, C_gt, pairs.to(device), npairs, a1, a2, o12, o21, t12, t21,
                                       selection=(rows, valid))
        loss.backward()
        res.append((float(loss), a1.grad.clone(), a2.grad.clone()))
    assert abs(res[0][0] - res[1][0]) <= 1e-5 * abs(res[0][0])
    for k in (1, 2):
        scale = float(res[0][k].abs().max())
        assert (res[0][k] - res[1][k]).abs().max().item() <= 1e-5 * scale, k


@pytest.mark.parametrize("N1,N2", [(256, 256), (300, 200)])
def test_fused_fmap_head_matches_module_path(device, N1, N2, monkeypatch):
    """DPFMNet with the fused fmap head (pk_fmap_head_fwd / _bwd around the solve) against
    the module path (evecs_trans products, batched GEMMs, resolvent mask, solve) on the same
    weights and inputs: C_pred within 1e-4 of its scale and the parameter gradients within
    1e-3 in norm (f32 summation order of the projections differs, and the lambda = 100
    regularized solve amplifies it; test_dpfmnet_matches_oracle holds the fused path to the
    fp64 oracle with the 3x fp32 yardstick, parameter by parameter)."""
    from dpfm_amd.models import dpfm as MD
    from dpfm_amd.models.dpfm import DPFMNet
    torch.manual_seed(21)
    net = DPFMNet().to(device)
    b = _to(_inputs(2, N1, N2, seed=5), device)
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setattr(MD, "FUSED_FMAP_HEAD", mode == "1")
        net.zero_grad(set_to_none=True)
        C = net(b)[0]
        g = torch.linspace(-1, 1, C.numel(), device=device).view_as(C)
        (C * g).sum().backward()
        res[mode] = (C.detach().clone(), {k: p.grad.detach().clone() for k, p in net.named_parameters()
                                          if p.grad is not None})
    sc = float(res["0"][0].abs().max())
    assert (res["1"][0] - res["0"][0]).abs().max().item() <= 1e-4 * sc
    assert res["1"][1].keys() == res["0"][1].keys()
    # all parameter gradients together (single small gradients, e.g. the merge bias's
    # near-cancelling point sum, differ relatively more; test_dpfmnet_matches_oracle holds each
    # parameter of the fused path to the fp64 oracle)
    g0 = torch.cat([g.reshape(-1) for g in res["0"][1].values()])
    g1 = torch.cat([res["1"][1][k].reshape(-1) for k in res["0"][1]])
    assert (g1 - g0).norm().item() <= 1e-3 * g0.norm().item()


@pytest.mark.parametrize("N1,N2,layers,pair", [(512, 384, 1, True), (300, 203, 1, True), (300, 203, 2, True),
                                                (512, 384, 2, False)])  # (300, 203): ragged channels-first tiles
def test_fused_attn_prop_matches_module_path(device, monkeypatch, N1, N2, layers, pair):
    """attnprop._AttnPropPairFn (both calls of a refinement layer as one autograd node: the two
    gradients that meet at desc0' and at desc1 summed in launch epilogues) and _AttnPropFn (one
    node per AttentionalPropagation call + residual: stacked key/value projection, attention on
    the stacked buffer, merge into the concatenation, the input gradients of desc summed in one
    epilogue) vs the module path (modeling/dpfm.py:45-82, 101-103): refinement outputs and every
    parameter gradient within fp32 rounding (1e-5 of each tensor's scale; the summation orders
    differ)."""
    from dpfm_amd import attnprop
    from dpfm_amd.modeling import dpfm as MD
    if not pair:
        monkeypatch.setattr(attnprop, "attn_prop_pair", lambda *a: None)
    torch.manual_seed(3)
    net = MD.CrossAttentionRefinementNet(n_in=32, num_head=2, gnn_dim=32, n_layers=layers,
                                         cross_sampling_ratio=1).to(device)
    g = torch.Generator().manual_seed(4)
    fx = torch.randn(4, N1, 32, generator=g).to(device)
    fy = torch.randn(4, N2, 32, generator=g).to(device)

    def run(fused):
        monkeypatch.setattr(MD, "FUSED_ATTN_PROP", fused)
        net.zero_grad()
        a, b = fx.clone().requires_grad_(True), fy.clone().requires_grad_(True)
        rx, ry, ox, oy = net(None, None, a, b)
        (rx.square().sum() + 0.5 * ry.square().sum() + ox.sum() + 2 * oy.sum()).backward()
        return [t.detach().clone() for t in (rx, ry, ox, oy, a.grad, b.grad)] + \
               [p.grad.detach().clone() for p in net.parameters()]

    ref, got = run(False), run(True)
    names = ["rx", "ry", "ox", "oy", "dfx", "dfy"] + [n for n, _ in net.named_parameters()]
    # floor for parameters whose true gradient vanishes by invariance (biases in front of the
    # InstanceNorm: merge / mlp.0 biases): their values are rounding noise of the global scale
    floor = 1e-6 * float(torch.cat([r.reshape(-1) for r in ref[6:]]).norm())
    for n, r, o in zip(names, ref, got):
        scale = max(float(r.abs().max()), 1e-30)
        assert (o - r).abs().max().item() <= 1e-5 * scale + floor, (n, (o - r).abs().max().item(), scale, floor)

def test_first_lin_pair_matches_per_shape(device):
    """layers._LinearPairCfFn (the refinement's first_lin once over the encoder's concatenated
    [2B, N, C] features, channels-first output, the two gradients transposed into one rows dy by
    pk_transpose_cf_rows) vs first_lin per shape (modeling/dpfm.py:98): refinement outputs, the
    features' gradient and every parameter gradient within fp32 rounding."""
    from dpfm_amd.modeling import dpfm as MD
    torch.manual_seed(5)
    net = MD.CrossAttentionRefinementNet(n_in=32, num_head=2, gnn_dim=32, n_layers=2, cross_sampling_ratio=1).to(device)
    g = torch.Generator().manual_seed(6)
    feat = torch.randn(6, 300, 32, generator=g).to(device)

    def run(pair):
        net.zero_grad()
        f = feat.clone().requires_grad_(True)
        fx, fy = torch.chunk(f, 2, 0)
        rx, ry, ox, oy = net(None, None, fx, fy, features_xy=f if pair else None)
        (rx.square().sum() + 0.5 * ry.square().sum() + ox.sum() + 2 * oy.sum()).backward()
        return [t.detach().clone() for t in (rx, ry, ox, oy, f.grad)] + [p.grad.detach().clone() for p in net.parameters()]

    ref, got = run(False), run(True)
    floor = 1e-6 * float(torch.cat([r.reshape(-1) for r in ref[5:]]).norm())
    for i, (r, o) in enumerate(zip(ref, got)):
        scale = max(float(r.abs().max()), 1e-30)
        assert (o - r).abs().max().item() <= 1e-5 * scale + floor, (i, (o - r).abs().max().item(), scale)


@pytest.mark.parametrize("N", [1024, 300])  # 300: ragged channels-first tiles (SUB = 1)
def test_linear_ex2_pair_matches_two_calls(device, N):
    """pk_linear_ex2 (two independent channels-first layers in one launch) writes exactly what
    two pk_linear_ex calls write, for every Cin / Cout pair it takes and the epilogues the
    refinement uses (bias, stacked weight + bias2, transposed weight, add, add2)."""
    from dpfm_amd import ops
    g = torch.Generator().manual_seed(8)
    B = 32 if N == 1024 else 4  # 32 x 1024: 32 points per wave (SUB = 2)

    def r(*s):
        return torch.randn(*s, generator=g).to(device)

    for ci0, co0, ci1, co1 in [(32, 32, 32, 64), (32, 32, 64, 32), (64, 64, 32, 32), (64, 32, 64, 64)]:
        x0, x1 = r(B, ci0, N), r(B, ci1, N)
        w0, w1, b0, b1 = r(co0, ci0), r(co1 // 2, ci1), r(co0), r(co1 // 2)
        w1b, b1b = r(co1 - co1 // 2, ci1), r(co1 - co1 // 2)
        add0, add20 = r(B, co0, N), r(B, co0, N)
        kw0 = dict(add=add0, add_cols=co0, add2=add20)
        kw1 = dict(w2=w1b, bias2=b1b, wsplit=co1 // 2)
        outs = []
        for pair in (False, True):
            y0, y1 = torch.full((B, co0, N), 7.0, device=device), torch.full((B, co1, N), 7.0, device=device)
            a0 = (x0, w0, b0, 1, B * N, N, ci0, co0, y0)
            a1 = (x1, w1, b1, 1, B * N, N, ci1, co1, y1)
            if pair:
                ops.linear_ex2(a0, kw0, a1, kw1)
            else:
                ops.linear_ex(*a0, **kw0)
                ops.linear_ex(*a1, **kw1)
            outs.append((y0.cpu(), y1.cpu()))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), (ci0, co0, ci1, co1)
        ref0 = torch.einsum("oi,bin->bon", w0.cpu(), x0.cpu()) + b0.cpu()[None, :, None] + add0.cpu() + add20.cpu()
        assert (outs[1][0] - ref0).abs().max().item() <= 1e-4 * ref0.abs().max().item()
