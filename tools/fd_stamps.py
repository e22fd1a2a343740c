"""Phase stamps of the feature-distance main pass (dev library, PK_FD_VAR=13). Top-1: per block
the s_memtime at kernel entry (0), after the prologue operands arrived (1), after the main loop
(2), after the per-column reductions (3), at exit (4), and the HW_ID / XCC_ID registers (5, 6).
Top-5: entry (0), staging (1), main loop (2), E0+E1 (3), E2 (4), E3 (5), E3b (6), E3c's task
merge (8) and list merges (9), emit + barrier (10), slow path + exit (7); slow columns (11) and
recompute rows (12) per block. Prints the phase durations (cycles, median / p90 / max over blocks).
   PK_DEV=1 PK_FD_VAR=13 python tools/fd_stamps.py [BxV] [topk]"""
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
topk = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda:0")
ex = torch.stack([torch.from_numpy(lbo_operators(V, 64, 10 + b)[2]) for b in range(B)]).to(dev)
ey = torch.stack([torch.from_numpy(lbo_operators(V, 64, 50 + b)[2]) for b in range(B)]).to(dev)
C = (torch.eye(30)[None] + 0.3 * torch.randn(B, 30, 30, generator=torch.Generator().manual_seed(B))).to(dev)
n = torch.full((B,), V, dtype=torch.int32, device=dev)
for _ in range(50):
    ops.feat_dist_topk(ex, C, ey, n, n, topk)
torch.cuda.synchronize()
NB = 4096
buf = (ctypes.c_ulonglong * (NB * 16))()
_lib.dev_lib().pkdev_fd_stamps(buf, NB * 16)
st = np.frombuffer(buf, dtype=np.uint64).reshape(NB, 16).astype(np.int64)
nb = int((st[:, 0] != 0).sum())
st = st[:nb]
if topk == 5:
    names = ["staging 0-1", "main loop 1-2", "E0+E1 2-3", "E2 3-4", "E3 scan 4-13", "E3 merges 13-14",
             "E3 list+sync 14-5", "E3b 5-6", "E3c 6-8", "emit+sync 9-10", "slow 10-7", "total 0-7"]
    pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 13), (13, 14), (14, 5), (5, 6), (6, 8), (9, 10), (10, 7), (0, 7)]
else:
    names = ["prologue 0-1", "main loop 1-2", "reductions 2-3", "merge+store 3-4", "total 0-4"]
    pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (0, 4)]
print(f"{shape} top-{topk}: {nb} blocks (s_memtime: shader clock cycles)")
for nm, (a, b) in zip(names, pairs):
    d = st[:, b] - st[:, a]
    print(f"  {nm:16s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  max {d.max():8d}  min {d.min():8d}")
if topk == 5:
    print(f"  slow columns per block: mean {st[:, 11].mean():.2f} max {st[:, 11].max()}; "
          f"recompute rows per block: mean {st[:, 12].mean():.1f} max {st[:, 12].max()}")
    sys.exit(0)
hw = st[:, 5]
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
xcc = st[:, 6] & 0xF
key = list(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
cnt = Counter(key)
print(f"  distinct CUs {len(cnt)}; blocks per CU histogram {sorted(Counter(cnt.values()).items())}")
print(f"  simd ids {sorted(Counter(((hw >> 4) & 3).tolist()).items())}")
