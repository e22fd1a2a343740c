"""SOR alone on the bench's crop-formation input (development aid for counter runs)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch
from dpfm_amd import ops
from dpfm_amd.pipeline import make_frame_batch

dev = torch.device("cuda:0")
fb, _ = make_frame_batch(32, 1024, 1024, seed=0, device=dev)
bp = ops.backproject(fb.depth, fb.mask, fb.K, fb.cam_scale, cap=32 * fb.max_pixels)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    ops.sor(bp["xyz"], bp["off"], fb.max_pixels, 20, 0.3, pix=bp["pix"], idxmap=bp["idxmap"], K=fb.K)
torch.cuda.synchronize()
