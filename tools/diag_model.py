"""Dev diagnostic: per-parameter gradient error vs the fp64 oracle for (a) the oracle in
fp32 on the CPU, (b) the oracle in fp32 with torch on the GPU, (c) the HIP path."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from oracle import dpfm_model_oracle as M  # noqa: E402
from test_model_gpu import _inputs, _to  # noqa: E402
from dpfm_amd.models.dpfm import DPFMNet  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(3)
ref = M.DPFMNet()
with torch.no_grad():
    ref.feature_extractor.block_0.diffusion.diffusion_time.uniform_(-0.001, 12)
    ref.feature_extractor.block_1.diffusion.diffusion_time.uniform_(-0.001, 12)
truth = M.DPFMNet().double()
truth.load_state_dict(ref.state_dict())
gref = M.DPFMNet().to(dev)
gref.load_state_dict(ref.state_dict())
mine = DPFMNet().to(dev)
mine.load_state_dict(ref.state_dict())
batch = _inputs(2, 256, 256, seed=5)
b64 = {k: {kk: vv.double() for kk, vv in v.items()} for k, v in batch.items()}
models = [(truth, b64), (ref, batch), (gref, _to(batch, dev)), (mine, _to(batch, dev))]
for lname, lf in (("feat", lambda o: o[1].sum() + o[2].sum() + o[3].square().sum() + o[4].square().sum()),
                  ("C", lambda o: o[0].sum())):
    grads = []
    for m, bt in models:
        m.zero_grad()
        lf(m(bt)).backward()
        grads.append([torch.zeros_like(p).cpu().double() if p.grad is None else p.grad.detach().cpu().double()
                      for p in m.parameters()])
    print(f"== loss {lname}: rel Frobenius error vs fp64   cpu32   gpu-torch32   hip")
    for i, (name, _) in enumerate(truth.named_parameters()):
        t = grads[0][i]
        nt = t.norm().item() + 1e-30
        e = [(g[i] - t).norm().item() / nt for g in grads[1:]]
        print(f"{name:60s} {e[0]:.2e} {e[1]:.2e} {e[2]:.2e}")
