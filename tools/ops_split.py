"""(f1) where the operator time goes: geometry.get_operators on bench.py's operators workload
(B crops x N points, k = 64) with robust=True (tufted-cover intrinsic-Delaunay flips on host
threads, robust_laplacian's operator) and robust=False (the fan soup's own cotan Laplacian: the
same device kNN / fans / eigensolver, no host stage), plus the host stage alone (tufted_dense).

  python tools/ops_split.py [B] [N]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dpfm_amd import geometry, ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
dev = torch.device("cuda:0")
shapes = bench.ops_workload(B, N, 0)


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


t_rob = timed(lambda: geometry.get_operators(shapes, k_eig=64, device=dev))
t_soup = timed(lambda: geometry.get_operators(shapes, k_eig=64, device=dev, robust=False))
pts, off, nmax = geometry._pack(shapes, dev)
counts = [int(s.shape[0]) for s in shapes]
idx, _ = ops.knn(pts, off, nmax, 30, omit_self=True)
tri, ntri, _ = ops.pc_local_tri(pts, off, nmax, idx)
t_flip = timed(lambda: geometry.tufted_dense(pts, off, counts, nmax, tri, ntri))
print(f"operators B={B} N={N} k=64: robust (tufted flips) {t_rob * 1e3:.1f} ms = {B / t_rob:.1f} sets/s; "
      f"fan soup (no flips) {t_soup * 1e3:.1f} ms = {B / t_soup:.1f} sets/s; host tufted stage alone "
      f"{t_flip * 1e3:.1f} ms ({t_flip / t_rob:.0%} of the robust batch, {min(B, 16)} host threads)")
