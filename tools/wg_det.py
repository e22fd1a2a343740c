"""Grouped weight gradients: run-to-run bit equality and the fp64 error bound on the training step's
call list (tools/wg_bench.py's shapes) plus ragged / small problems, under the block budget in
PK_WG_BUDGET (dev library). Prints the first mismatching call, if any.

  PK_WG_BUDGET=1024 python tools/wg_det.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

from dpfm_amd import _lib, ops  # noqa: E402

_lib.use_dev_lib()
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1)
spec = [("cf", (32, 32, 1024), 32, 4), ("cf", (32, 64, 1024), 64, 1), ("cl", (32768, 32), 1, 1),
        ("cl", (32768, 32), 32, 2), ("cl", (65536, 128), 64, 1), ("cl", (65536, 3), 64, 1),
        ("cl", (65536, 64), 64, 2), ("cl", (165, 64), 32, 1), ("cl", (4004, 32), 1, 1), ("cf", (3, 64, 2000), 64, 1),
        ("cf", (2, 32, 48), 32, 1), ("cl", (20, 128), 64, 1)]
calls, refs = [], []
for lay, xs, O, cnt in spec:
    for _ in range(cnt):
        x = torch.randn(*xs, device=dev, generator=g)
        if lay == "cf":
            Bn, I, N = xs
            dy = torch.randn(Bn, O, N, device=dev, generator=g)
            ew = torch.einsum("bon,bin->oi", dy.double(), x.double())
            bw = torch.einsum("bon,bin->oi", dy.double().abs(), x.double().abs())
        else:
            R, I = xs
            dy = torch.randn(R, O, device=dev, generator=g)
            ew, bw = dy.double().t() @ x.double(), dy.double().abs().t() @ x.double().abs()
        calls.append((x, dy, lay == "cf", torch.full((O, I), float("nan"), device=dev),
                      torch.full((O,), float("nan"), device=dev), False))
        refs.append((ew, bw))
outs = []
for rep in range(3):
    for c in calls:
        c[3].fill_(float("nan"))
        c[4].fill_(float("nan"))
    ops.linear_wgrad_grouped(calls)
    torch.cuda.synchronize()
    outs.append([c[3].clone() for c in calls])
bad = 0
for i, ((ew, bw), c) in enumerate(zip(refs, calls)):
    same = all(torch.equal(outs[0][i], outs[r][i]) for r in range(1, 3))
    ok = bool((outs[0][i].double() - ew).abs().le(1e-5 * bw + 1e-30).all())
    if not (same and ok):
        bad += 1
        print(f"call {i} ({tuple(c[0].shape)} -> {c[3].shape[0]}, cf={c[2]}): repeatable={same} within_bound={ok} "
              f"nan={int(torch.isnan(outs[0][i]).sum())}")
print(f"budget {os.environ.get('PK_WG_BUDGET', 'default')}: {len(calls)} calls, {bad} bad")
