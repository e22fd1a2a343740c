"""Per-wave phase cycles of the flat FPS kernel (dev library, pkdev_fps_cfg pruned=6): for each of
the 16 waves of a crop's workgroup, s_memtime cycles per iteration spent in (read of the centroid +
box test), (update + wave reduction, counted only on updating iterations) and (atomic + barrier), and
the fraction of iterations the wave updated. Crops as tools/kbench.py: B = 32 synthetic frames.
   python tools/fps_stamps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dpfm_amd import _lib, ops  # noqa: E402

_lib.use_dev_lib()
from dpfm_amd.pipeline import make_frame_batch  # noqa: E402

dev = torch.device("cuda:0")
B, npt = 32, 1024
fb, _ = make_frame_batch(B, 1024, 1024, seed=0, device=dev)
bp = ops.backproject(fb.depth, fb.mask, fb.K, fb.cam_scale, cap=B * fb.max_pixels)
so = ops.sor(bp["xyz"], bp["off"], fb.max_pixels, 20, 0.3, pix=bp["pix"], idxmap=bp["idxmap"], K=fb.K)
x, off = so["xyz32"], so["off"]
nin = int((off[1:] - off[:-1]).max())
st = torch.zeros(B, dtype=torch.int32, device=dev)
npv = torch.full((B,), npt, dtype=torch.int32, device=dev)
ref = ops.fps_packed(x, off, nin, st, npv, npt)
out = torch.zeros((B, npt), dtype=torch.int64, device=dev)
L = _lib.lib()
for _ in range(20):
    rc = L.pkdev_fps_cfg(_lib.ptr(x), _lib.ptr(off), B, nin, _lib.ptr(st), _lib.ptr(npv), _lib.ptr(out), npt, 1024, 6,
                         _lib.stream(dev))
    assert rc == 0, rc
torch.cuda.synchronize()
print(f"B={B} n_in<={nin} npoint={npt}: same as production = {torch.equal(out, ref)}")
N = 64 * 16 * 8
buf = (ctypes.c_ulonglong * N)()
_lib.dev_lib().pkdev_fps_stamps(buf, N)
a = np.frombuffer(buf, dtype=np.uint64).reshape(64, 16, 8).astype(np.float64)[:B]
it = a[:, :, 4]
box, upd, bar, nupd = a[:, :, 0] / it, a[:, :, 1], a[:, :, 2] / it, a[:, :, 3]
updper = np.where(nupd > 0, upd / np.maximum(nupd, 1), 0)
tot = (a[:, :, 0] + a[:, :, 1] + a[:, :, 2]) / it
print("cycles per iteration, mean over crops, per wave (w0..w15):")
for nm, v in [("read+box", box), ("update (per updating it)", updper), ("update (per it)", upd / it),
              ("atomic+barrier", bar), ("updating fraction", nupd / it), ("total", tot)]:
    print(f"  {nm:26s} " + " ".join(f"{x:6.0f}" if nm != "updating fraction" else f"{x:6.2f}" for x in v.mean(0)))
print(f"per crop total cycles/iteration: median {np.median(tot[:, 0]):.0f}; "
      f"min wave barrier wait per it: median {np.median(bar.min(1)):.0f}")
