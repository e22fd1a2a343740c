"""Which kernel dominates the gradient error of DPFMNet on real crops (N1 = 5002, N2 = 2000)?
Runs the fmap-path gradient (o[0].sum()) of the HIP model with one fused op at a time swapped
for its plain-torch form, and prints each parameter's error vs the fp64 oracle.
  python tools/diag_real_grad.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import dpfm_model_oracle as M  # noqa: E402
from dpfm_amd import ops  # noqa: E402
from dpfm_amd.models.dpfm import DPFMNet  # noqa: E402
from test_ragged_gpu import _real_batch  # noqa: E402

dev = torch.device("cuda:0")
_, batch = _real_batch([0, 3, 6])
batch = {k: {kk: vv for kk, vv in v.items() if kk in ("xyz", "mass", "evals", "evecs")} for k, v in batch.items()}
torch.manual_seed(7)
ref = M.DPFMNet()
with torch.no_grad():
    ref.feature_extractor.block_0.diffusion.diffusion_time.uniform_(-0.001, 12)
    ref.feature_extractor.block_1.diffusion.diffusion_time.uniform_(-0.001, 12)
truth = M.DPFMNet().double()
truth.load_state_dict(ref.state_dict())
b64 = {k: {kk: vv.double() for kk, vv in v.items()} for k, v in batch.items()}
bdev = {k: {kk: vv.to(dev) for kk, vv in v.items()} for k, v in batch.items()}


def grads(m, b, fn):
    m.zero_grad()
    fn(m(b)).backward()
    return {n: (p.grad.detach().cpu().double() if p.grad is not None else torch.zeros(p.shape, dtype=torch.float64))
            for n, p in m.named_parameters()}


FN = {"fmap": lambda o: o[0].sum(), "feat": lambda o: o[1].sum() + o[2].sum() + o[3].square().sum() + o[4].square().sum()}
T = {k: grads(truth, b64, f) for k, f in FN.items()}
gref = M.DPFMNet().to(dev)
gref.load_state_dict(ref.state_dict())
R = {k: grads(gref, bdev, f) for k, f in FN.items()}
C = {k: grads(ref, batch, f) for k, f in FN.items()}


def torch_attention(q, k, v):
    s = torch.einsum("bdhn,bdhm->bhnm", q, k) / q.shape[1] ** 0.5
    return torch.einsum("bhnm,bdhm->bdhn", torch.softmax(s, -1), v)


def torch_spectral(x, mass, evals, evecs, t):
    spec = torch.matmul(evecs.transpose(-2, -1), x * mass.unsqueeze(-1))
    return torch.matmul(evecs, torch.exp(-evals.unsqueeze(-1) * t.unsqueeze(0)) * spec)


def torch_instnorm(x, eps=1e-5):
    return torch.relu(F.instance_norm(x, eps=eps))


def torch_fmap(AAt, BAt, D, lam):
    rows = [torch.linalg.solve(AAt + lam * torch.diag_embed(D[:, i, :]), BAt[:, i, :, None]).transpose(1, 2)
            for i in range(AAt.shape[1])]
    return torch.cat(rows, 1)


SWAPS = {"none": {}, "attention": {"attention": torch_attention}, "spectral": {"spectral_diffusion": torch_spectral},
         "instnorm": {"instnorm_relu": torch_instnorm}, "fmap_solve": {"fmap_solve": torch_fmap},
         "l2norm": {"l2_normalize": lambda x: F.normalize(x, p=2, dim=-1)}}
orig = {k: getattr(ops, k) for s in SWAPS.values() for k in s}
for name, sw in SWAPS.items():
    for k, f in sw.items():
        setattr(ops, k, f)
    mine = DPFMNet().to(dev)
    mine.load_state_dict(ref.state_dict())
    for key, fn in FN.items():
        G = grads(mine, bdev, fn)
        worst = []
        for p in T[key]:
            t = T[key][p]
            e = [(x[p] - t).norm().item() for x in (C[key], R[key], G)]
            worst.append((e[2] / max(e[0], e[1], 1e-30), p, e, t.norm().item()))
        worst.sort(reverse=True)
        print(f"[{name:10s}] {key}: worst ratio {worst[0][0]:.2f} {worst[0][1]} {worst[0][2]} |g|={worst[0][3]:.3g};"
              f" 2nd {worst[1][0]:.2f} {worst[1][1]}", flush=True)
    for k in sw:
        setattr(ops, k, orig[k])
