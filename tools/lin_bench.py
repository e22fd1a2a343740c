"""Device time per pk_linear_fwd launch for the model's shapes (50 launches captured in a
HIP graph and replayed, so host launch overhead is off the clock), vs the HBM ideal."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch
from dpfm_amd import _lib, ops

if os.environ.get("PK_DEV") == "1":  # libposekern_dev.so (its PK_* switches, e.g. PK_ROWS_GLDS=0)
    _lib.use_dev_lib()

dev = torch.device("cuda:0")
shapes = [  # (lead, Cin, Cout, cf, transw)  lead = rows (cl) or (B, N) (cf)
    (65536, 128, 64, False, False), (65536, 64, 64, False, False), (65536, 3, 64, False, False),
    (65536, 64, 32, False, False), (65536, 64, 128, False, True), (65536, 64, 64, False, True),
    (65536, 32, 64, False, True), ((32, 1024), 32, 32, True, False), ((32, 1024), 64, 64, True, False),
    ((32, 1024), 64, 32, True, False), ((32, 1024), 32, 64, True, True), ((32, 1024), 32, 1, True, False), ((32, 1024), 1, 32, True, True), (65536, 32, 1, False, False),
]
for lead, ci, co, cf, tw in shapes:
    if cf:
        B, N = lead
        x = torch.randn(B, ci, N, device=dev)
        R = B * N
    else:
        x = torch.randn(lead, ci, device=dev)
        R = lead
    w = torch.randn(ci, co, device=dev) if tw else torch.randn(co, ci, device=dev)
    b = None if tw else torch.randn(co, device=dev)
    f = lambda: ops.linear_fwd(x, w, b, channels_first=cf, transw=tw)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(50):
                f()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    byts = 4.0 * R * (ci + co)
    print(f"R={R} {ci}->{co} {'cf' if cf else 'cl'}{' T' if tw else ''}: {us:6.1f} us  {byts/us/1e3:6.0f} GB/s  "
          f"ideal {byts/8e12*1e6:5.1f} us  {2*R*ci*co/us/1e6:6.1f} TF/s", flush=True)

# the diffusion-net block's pk_linear_ex launches as the training step issues them (R = 2 x 32 x 1024)
R = 65536
cat = torch.randn(R, 128, device=dev)
h = torch.randn(R, 64, device=dev)
m = torch.rand(R, 64, device=dev) - 0.5
w1, w2, w3 = torch.randn(64, 128, device=dev), torch.randn(64, 64, device=dev), torch.randn(64, 64, device=dev)
b = torch.randn(64, device=dev)
o64, o64b, o128 = torch.empty(R, 64, device=dev), torch.empty(R, 64, device=dev), torch.empty(R, 128, device=dev)
cases = [
    ("fwd 128->64 relu", lambda: ops.linear_ex(cat, w1, b, 0, R, 0, 128, 64, y=o64, relu=True), 128 + 64),
    ("fwd 64->64 relu", lambda: ops.linear_ex(h, w2, b, 0, R, 0, 64, 64, y=o64, relu=True), 128),
    ("fwd 64->64 +res ldy128", lambda: ops.linear_ex(h, w3, b, 0, R, 0, 64, 64, y=o128, ldy=128, add=cat, lda=128,
                                                    add_cols=64), 192),
    ("bwd 64->64 T mask", lambda: ops.linear_ex(h, w3, None, 0, R, 0, 64, 64, y=o64, transw=True, mask=m), 192),
    ("bwd 64->128 T split+add", lambda: ops.linear_ex(h, w1, None, 0, R, 0, 64, 128, y=o64, transw=True, y2=o64b,
                                                      split=64, add=m, add_cols=64), 256),
]
for name, f, bpr in cases:
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(50):
                f()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    print(f"{name}: {us:6.1f} us  {4.0 * R * bpr / us / 1e3:6.0f} GB/s", flush=True)
