"""Feature-distance + argmin / top-5 (pk_feat_dist_topk) at the BASELINE shapes, timed in
HIP graphs (no host gaps): configs[1] (32 crops of 1024 x 1024) and configs[4] (one 4096 x
4096 crop), every precision mode. Prints achieved TFLOP/s and, for the bf16 modes, the
argmin / top-5 agreement with the fp32 path.

  python tools/fd_bench.py [iters] [BxV] [precisions, comma-separated] [top-k values, comma-separated]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

from dpfm_amd import _lib, ops  # noqa: E402

if os.environ.get("PK_DEV") == "1":  # libposekern_dev.so (its PK_FD_* switches)
    _lib.use_dev_lib()
from dpfm_amd.dataset.synthetic import lbo_operators  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
only = sys.argv[2] if len(sys.argv) > 2 else None  # e.g. "32x1024"
precs = sys.argv[3].split(",") if len(sys.argv) > 3 else ["fp32", "bf16x3", "bf16"]
warm = int(os.environ.get("FD_WARM", "100"))  # untimed graph replays before timing
dev = torch.device("cuda:0")
for B, V in [(32, 1024), (8, 2048), (1, 4096)]:
    if only and only != f"{B}x{V}":
        continue
    ex = torch.stack([torch.from_numpy(lbo_operators(V, 64, 10 + b)[2]) for b in range(B)]).to(dev)
    ey = torch.stack([torch.from_numpy(lbo_operators(V, 64, 50 + b)[2]) for b in range(B)]).to(dev)
    C = (torch.eye(30)[None] + 0.3 * torch.randn(B, 30, 30, generator=torch.Generator().manual_seed(B))).to(dev)
    n = torch.full((B,), V, dtype=torch.int32, device=dev)
    ref = {}
    topks = tuple(int(x) for x in sys.argv[4].split(",")) if len(sys.argv) > 4 else ((1,) if only else (1, 5))
    for topk in topks:
        for prec in precs:
            wk = torch.zeros(1 << 24, dtype=torch.uint8, device=dev)  # one zeroed scratch, reused
            f = lambda: ops.feat_dist_topk(ex, C, ey, n, n, topk, precision=prec, work=wk)  # noqa: E731
            for _ in range(3):
                out = f()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(iters):
                    f()
            for _ in range(warm):  # past the clock ramp (profiles/r06_bq_ramp.txt)
                gr.replay()
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for e0, e1 in evs:
                e0.record()
                gr.replay()
                e1.record()
            torch.cuda.synchronize()
            ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs)[2] / iters  # median of 5 replays
            fl = 2.0 * B * V * V * 32
            peak = 157.3 if prec == "fp32" else 2500.0
            idx = out[0]
            if prec == "fp32" or topk not in ref:
                ref[topk] = idx
                agree = ""
            else:
                a1 = (idx[..., 0] == ref[topk][..., 0]).float().mean().item()
                agree = f", first-choice agreement with fp32 {a1:.4f}"
                if topk == 5:
                    same = (idx.sort(-1).values == ref[5].sort(-1).values).all(-1).float().mean().item()
                    agree += f", same top-5 set {same:.4f}"
            print(f"feat_dist_topk B={B} V={V} topk={topk} {prec}: {ms * 1e3:.1f} us/launch (prep + main), "
                  f"{fl / ms / 1e9:.1f} TFLOP/s = {fl / ms / 1e9 / peak:.3f} of the {'f32' if prec == 'fp32' else 'bf16'}"
                  f" MFMA peak{agree}", flush=True)

