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
