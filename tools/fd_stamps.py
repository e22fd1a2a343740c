"""Phase stamps of the top-1 feature-distance pass (dev library, PK_FD_VAR=13): per block the
s_memtime at kernel entry (0), after the prologue operands arrived (1), after the main loop (2),
after the per-column reductions (3), at exit (4), and the HW_ID / XCC_ID registers (5, 6).
Prints the phase durations (cycles, median / p90 / max over blocks) and how many blocks shared a
CU.   PK_DEV=1 PK_FD_VAR=13 python tools/fd_stamps.py [BxV]"""
import ctypes
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dpfm_amd import _lib, ops  # noqa: E402

_lib.use_dev_lib()
from dpfm_amd.dataset.synthetic import lbo_operators  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "32x1024"
B, V = map(int, shape.split("x"))
dev = torch.device("cuda:0")
ex = torch.stack([torch.from_numpy(lbo_operators(V, 64, 10 + b)[2]) for b in range(B)]).to(dev)
ey = torch.stack([torch.from_numpy(lbo_operators(V, 64, 50 + b)[2]) for b in range(B)]).to(dev)
C = (torch.eye(30)[None] + 0.3 * torch.randn(B, 30, 30, generator=torch.Generator().manual_seed(B))).to(dev)
n = torch.full((B,), V, dtype=torch.int32, device=dev)
for _ in range(50):
    ops.feat_dist_topk(ex, C, ey, n, n, 1)
torch.cuda.synchronize()
NB = 4096
buf = (ctypes.c_ulonglong * (NB * 8))()
_lib.dev_lib().pkdev_fd_stamps(buf, NB * 8)
st = np.frombuffer(buf, dtype=np.uint64).reshape(NB, 8).astype(np.int64)
nb = int((st[:, 0] != 0).sum())
st = st[:nb]
names = ["prologue 0-1", "main loop 1-2", "reductions 2-3", "merge+store 3-4", "total 0-4"]
pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (0, 4)]
print(f"{shape}: {nb} blocks")
for nm, (a, b) in zip(names, pairs):
    d = st[:, b] - st[:, a]
    print(f"  {nm:16s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  max {d.max():8d}  min {d.min():8d}")
hw = st[:, 5]
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
xcc = st[:, 6] & 0xF
key = list(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
cnt = Counter(key)
print(f"  distinct CUs {len(cnt)}; blocks per CU histogram {sorted(Counter(cnt.values()).items())}")
print(f"  simd ids {sorted(Counter(((hw >> 4) & 3).tolist()).items())}")
