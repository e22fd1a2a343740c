"""Development timing of pk_nce_loss at the bench shape (B=32 crops, 1024 points, 512 pairs)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch
from dpfm_amd import ops

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
B, N, cap = 32, 1024, 4000
pairs = torch.stack([torch.randint(0, N, (B, cap), device=dev, generator=g),
                     torch.randint(0, N, (B, cap), device=dev, generator=g)], -1)
counts = torch.full((B,), cap, dtype=torch.int64, device=dev)
ctr = torch.zeros(1, dtype=torch.int64, device=dev)
rows, valid = ops.nce_select(counts, cap, 512, 3, ctr)
f1 = torch.randn(B, N, 32, device=dev, generator=g).requires_grad_(True)
f2 = torch.randn(B, N, 32, device=dev, generator=g).requires_grad_(True)
for mode in ("grad", "nograd"):
    def run():
        if mode == "grad":
            return ops.nce_loss(f1, f2, pairs, rows, valid, 0.07)
        with torch.no_grad():
            return ops.nce_loss(f1, f2, pairs, rows, valid, 0.07)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        run()
    e.record()
    torch.cuda.synchronize()
    print(mode, "ms/call", s.elapsed_time(e) / 20)
