"""The training step's attention shape (B = 32 crops, 2 heads, dim 16, N = M = 1024), forward +
backward through ops.attention, `reps` times eagerly (for rocprofv3 --pmc passes and kernel
traces): python tools/attn_pmc.py [reps]. Prints the per-launch time of each kernel family."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402
from dpfm_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, D, H, N = 32, 16, 2, 1024
g = torch.Generator(device=dev).manual_seed(0)
q, k, v = (torch.randn(B, D, H, N, device=dev, generator=g).requires_grad_() for _ in range(3))
do = torch.randn(B, D, H, N, device=dev, generator=g)


def step():
    o = ops.attention(q, k, v)
    return torch.autograd.grad(o, (q, k, v), do)


for _ in range(3):
    step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    step()
e1.record()
torch.cuda.synchronize()
fl = 2.0 * B * H * N * N * D
print(f"attention fwd+bwd {e0.elapsed_time(e1) * 1e3 / reps:.1f} us/iter (eager; {18 * fl / 1e9:.2f} GFLOP "
      f"incl. recomputation)", flush=True)
