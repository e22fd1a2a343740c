"""pk_spectral_diffusion (H7) timing at the training step's shapes: B crops x N points, K = C = 64,
forward (mode 0, mass-weighted reduce) and backward (mode 1, mass on the expand, accumulate),
graph-free back-to-back launches with HIP events; algorithmic bytes = Phi read twice + the
input rows + the output rows (+ the accumulated rows). With PK_DEV=1 the dev library is loaded
(PK_SPEC_SCALAR=1: round 1's scalar-FMA passes).

  python tools/spec_bench.py [B] [N]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

from dpfm_amd import _lib, ops  # noqa: E402

if os.environ.get("PK_DEV") == "1":
    _lib.use_dev_lib()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B, N, 128, device=dev, generator=g)  # a 64-wide slice of a concatenation buffer
mass = torch.rand(B, N, device=dev, generator=g)
evecs = torch.randn(B, N, 64, device=dev, generator=g) / N ** 0.5
evals = torch.rand(B, 64, device=dev, generator=g) * 10
t = torch.rand(64, device=dev, generator=g)
out = torch.empty(B, N, 128, device=dev)
gt = torch.empty(64, device=dev)


def fwd():
    return ops.spectral_raw(x, 128, mass, evals, evecs, t, False, 0, out[..., 64:], 128)


raw = fwd()


def bwd():
    ops.spectral_raw(x, 128, mass, evals, evecs, t, False, 1, out, 128, saved=raw, gt=gt, accumulate=True)


def timed(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


for name, fn, nb in (("forward", fwd, 4 * B * N * 64 * 4), ("backward", bwd, 4 * B * N * 64 * 5)):
    us = timed(fn)
    print(f"spectral {name} B={B} N={N} (3 launches): {us:6.1f} us  {nb / 1e6:5.1f} MB -> "
          f"{nb / us / 1e6:5.2f} TB/s ({nb / us / 1e6 / 8.0:.3f} of HBM)  "
          f"PK_SPEC_SCALAR={os.environ.get('PK_SPEC_SCALAR', '-')}")
