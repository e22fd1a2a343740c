"""One per-point layer shape of the training step, launched eagerly `reps` times (for
rocprofv3 --pmc passes and kernel traces): python tools/lin_pmc.py <case> [reps]."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402
from dpfm_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
case = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
R = 65536
g = torch.Generator(device=dev).manual_seed(0)
rnd = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
if case == "rows128_64":
    x, w, b, y = rnd(R, 128), rnd(64, 128), rnd(64), torch.empty(R, 64, device=dev)
    f = lambda: ops.linear_ex(x, w, b, 0, R, 0, 128, 64, y=y, relu=True)  # noqa: E731
elif case == "rows64_64_mask":
    x, w, b, y, m = rnd(R, 64), rnd(64, 64), rnd(64), torch.empty(R, 64, device=dev), rnd(R, 64)
    f = lambda: ops.linear_ex(x, w, None, 0, R, 0, 64, 64, y=y, transw=True, mask=m)  # noqa: E731
elif case == "cf32_32":
    B, N = 32, 1024
    x, w, b, y = rnd(B, 32, N), rnd(32, 32), rnd(32), torch.empty(B, 32, N, device=dev)
    f = lambda: ops.linear_ex(x, w, b, 1, B * N, N, 32, 32, y=y)  # noqa: E731
elif case == "cf64_64":
    B, N = 32, 1024
    x, w, b, y = rnd(B, 64, N), rnd(64, 64), rnd(64), torch.empty(B, 64, N, device=dev)
    f = lambda: ops.linear_ex(x, w, b, 1, B * N, N, 64, 64, y=y)  # noqa: E731
else:
    raise SystemExit(f"unknown case {case}")
for _ in range(reps):
    f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    f()
e1.record()
torch.cuda.synchronize()
print(case, f"{e0.elapsed_time(e1) * 1e3 / reps:.2f} us/launch (eager, back to back)", flush=True)
