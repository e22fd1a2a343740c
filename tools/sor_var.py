"""SOR time per call with a given libposekern build (variant A/B): python tools/sor_var.py lib.so [reps].
Prints the mean per-call device time (HIP events, 20 calls) and a checksum of the averages."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch
from dpfm_amd import _lib
_lib.LIB_PATH = os.path.abspath(sys.argv[1])
from dpfm_amd import ops
from dpfm_amd.pipeline import make_frame_batch

dev = torch.device("cuda:0")
fb, _ = make_frame_batch(32, 1024, 1024, seed=0, device=dev)
bp = ops.backproject(fb.depth, fb.mask, fb.K, fb.cam_scale, cap=32 * fb.max_pixels)
f = lambda: ops.sor(bp["xyz"], bp["off"], fb.max_pixels, 20, 0.3, pix=bp["pix"], idxmap=bp["idxmap"], K=fb.K)  # noqa: E731
out = f()
torch.cuda.synchronize()
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    f()
e1.record()
torch.cuda.synchronize()
keys = sorted(out.keys()) if isinstance(out, dict) else []
cs = {k: float(v.double().sum()) for k, v in out.items() if torch.is_tensor(v) and v.is_floating_point()} if keys else {}
print(os.path.basename(sys.argv[1]), f"{e0.elapsed_time(e1) / n * 1e3:.1f} us/call (sor entry)", cs, flush=True)
