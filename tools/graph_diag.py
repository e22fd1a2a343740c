"""Dev diagnostic: capture pieces of the training step into HIP graphs and compare each
replay with the eager result, from the safest piece to the riskiest; stop at the first
mismatch (nothing data-dependent runs on possibly-bad data).

  A  model forward (static crops)            B  forward + backward (sum-of-squares loss)
  C  crop formation (libposekern only)       D  full forward_backward (DPFM loss)
  E  D + clip + RMSprop
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] in ("cublas", "cublaslt"):
    torch.backends.cuda.preferred_blas_library(sys.argv[1])
print("blas:", torch.backends.cuda.preferred_blas_library(), flush=True)

from dpfm_amd.dataset.object import CropFormation  # noqa: E402
from dpfm_amd.models.dpfm import DPFMNet  # noqa: E402
from dpfm_amd.pipeline import TrainStep, model_batch, make_frame_batch  # noqa: E402

dev = torch.device("cuda:0")
F_, N = 4, 512
fb, op = make_frame_batch(F_, N, N, seed=90, device=dev)
cf = CropFormation(n1=N, npoint=N, seed=1)
crops = cf(fb)
torch.manual_seed(0)
model = DPFMNet().to(dev)


def capture(fn, warm=2):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def cmp(name, a, b, exact=False):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    fin = bool(torch.isfinite(b).all())
    d = (a - b).abs().max().item() if a.numel() else 0.0
    ok = fin and (d == 0.0 if exact else d <= 1e-4 * (1 + a.abs().max().item()))
    print(f"  {name}: max|diff| {d:.3e} finite={fin} {'OK' if ok else 'MISMATCH'}", flush=True)
    return ok


def stage(label, ok):
    print(f"{label}: {'PASS' if ok else 'FAIL'}", flush=True)
    if not ok:
        sys.exit(1)


# A: forward only
batch = model_batch(op, crops)
with torch.no_grad():
    ref = model(batch)
    g, out = capture(lambda: model(batch))
    g.replay()
    torch.cuda.synchronize()
    stage("A forward", all(cmp(f"out{i}", r, o) for i, (r, o) in enumerate(zip(ref[:5], out[:5]))))


# B: forward + backward with a plain loss
def fb_plain():
    o = model(batch)
    (o[0].square().sum() + o[1].sum() + o[2].sum() + o[3].square().sum() + o[4].square().sum()).backward()
    return [p.grad for p in model.parameters()]


model.zero_grad(set_to_none=True)
fb_plain()
ref = [p.grad.clone() for p in model.parameters()]
model.zero_grad(set_to_none=True)
g, grads = capture(lambda: (model.zero_grad(set_to_none=True), fb_plain())[1], warm=2)
g.replay()
torch.cuda.synchronize()
stage("B fwd+bwd", all(cmp(n, r, p.grad) for (n, p), r in zip(model.named_parameters(), ref)))

# C: crop formation
ref_c = cf(fb)
g, out_c = capture(lambda: cf(fb))
g.replay()
torch.cuda.synchronize()
okc = True
for name in ("pc64", "align64", "npairs", "overlap_12", "overlap_21", "off", "kept"):
    okc &= cmp(name, getattr(ref_c, name).double(), getattr(out_c, name).double(), exact=True)
# pair lists: only the first npairs[b] rows are written (the rest of the buffer is scratch)
cap = ref_c.pairs.shape[1]
valid = torch.arange(cap, device=dev)[None] < torch.clamp(ref_c.npairs, max=cap)[:, None]
okc &= cmp("pairs[:npairs]", (ref_c.pairs * valid[..., None]).double(), (out_c.pairs * valid[..., None]).double(),
           exact=True)
stage("C crop formation", okc)

# D / E: the real step (same RNG stream on both sides; warm-ups on a side stream)
for label, do_apply in (("D forward_backward", False), ("E + clip + RMSprop", True)):
    torch.manual_seed(0)
    m1 = DPFMNet().to(dev)
    m2 = DPFMNet().to(dev)
    m2.load_state_dict(m1.state_dict())
    s1, s2 = TrainStep(m1, seed=5, capturable=True), TrainStep(m2, seed=5, capturable=True)

    def run(st, reset):
        log = st.forward_backward(op, cf(fb))
        if do_apply:
            st.apply(allreduce=False, reset=reset)
        else:
            st.opt.zero_grad(set_to_none=reset)
        return log

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            run(s1, True)
            run(s2, True)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    g.register_generator_state(s2.gen)
    with torch.cuda.graph(g):
        log2 = run(s2, False)
    log1 = run(s1, True)
    g.replay()
    torch.cuda.synchronize()
    ok = cmp("loss", log1["loss"], log2["loss"]) and cmp("IR", log1["IR"], log2["IR"])
    stage(label, ok)
print("ALL PASS")
