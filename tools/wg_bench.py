"""Grouped weight gradients (pk_linear_wgrad_grouped) on the training step's call list at configs[1]
(tools/lin_census.py: 28 calls, 6.34 GFLOP), timed back to back with HIP events; prints us per
group, the algorithmic bytes (every x and dy read once) and FLOP rates against the MI355X peaks.
With PK_DEV=1 the dev library is loaded (PK_WG_GLDS=0: round 3's per-tile-wave kernel).

  python tools/wg_bench.py [iters] [--each]   (--each: every shape group alone as well)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

from dpfm_amd import _lib, ops  # noqa: E402

if os.environ.get("PK_DEV") == "1":
    _lib.use_dev_lib()

iters = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
# (layout, shape of x, O, count) as in the census of one training step
spec = [("cf", (32, 32, 1024), 32, 10), ("cf", (32, 64, 1024), 32, 2), ("cf", (32, 64, 1024), 64, 2),
        ("cl", (32768, 32), 1, 2), ("cl", (32768, 32), 32, 4), ("cl", (65536, 128), 64, 2),
        ("cl", (65536, 3), 64, 1), ("cl", (65536, 64), 32, 1), ("cl", (65536, 64), 64, 4)]
groups = []
calls, nbytes, flops = [], 0, 0
for lay, xs, O, cnt in spec:
    g0, b0, f0 = len(calls), nbytes, flops
    for _ in range(cnt):
        x = torch.randn(*xs, device=dev, generator=g)
        if lay == "cf":
            Bn, I, N = xs
            dy = torch.randn(Bn, O, N, device=dev, generator=g)
            R = Bn * N
        else:
            R, I = xs
            dy = torch.randn(R, O, device=dev, generator=g)
        dw = torch.empty(O, I, device=dev)
        db = torch.empty(O, device=dev)
        calls.append((x, dy, lay == "cf", dw, db, False))
        nbytes += 4 * R * (I + O)
        flops += 2 * R * I * O
    groups.append((f"{lay} {xs} -> {O} x{cnt}", calls[g0:], nbytes - b0, flops - f0))


def timed(cl):
    for _ in range(3):
        ops.linear_wgrad_grouped(cl)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.linear_wgrad_grouped(cl)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def line(name, us, nb, fl):
    return (f"{name:42s} {us:7.1f} us  {nb / 1e6:6.1f} MB -> {nb / us / 1e6:5.2f} TB/s ({nb / us / 1e6 / 8.0:.3f} "
            f"of HBM)  {fl / 1e9:5.2f} GFLOP -> {fl / us / 1e6:6.1f} TF/s ({fl / us / 1e6 / 157.3:.3f} of f32 MFMA)")


if os.environ.get("WG_ONLY"):  # one shape group alone (its index in spec), e.g. under rocprofv3
    name, calls, nbytes, flops = groups[int(os.environ["WG_ONLY"])]
    print(f"group {name}")
print(f"device: {torch.cuda.get_device_properties(0).multi_processor_count} CUs; "
      f"PK_WG_BUDGET={os.environ.get('PK_WG_BUDGET', '-')} PK_WG_GLDS={os.environ.get('PK_WG_GLDS', '-')}")
print("wgrad grouped " + line(f"({len(calls)} calls)", timed(calls), nbytes, flops))
if "--each" in sys.argv:
    for name, cl, nb, fl in groups:
        print("   " + line(name, timed(cl), nb, fl))
