"""pk_rigidity_filter A/B timing (pkdev_rigidity_variant): 0 the production path (grouped first
round, run-pair crop tables in rounds 2 / 3), 3 without the tables, 2 round 3's path (ungrouped
first round), 1 round 2's 64-tile gather path; B crops x n = 5 V2 candidates, eager back-to-back
launches; every variant's survivors compared with variant 0's.
RIGID_VARS=3,2,0 python tools/rigid_bench.py [V2 ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from dpfm_amd import _lib, ops  # noqa: E402
_lib.use_dev_lib()  # pkdev_* hooks: libposekern_dev.so (Makefile)
from test_configs_gpu import _rigid_scene  # noqa: E402

L = _lib.lib()
L.pkdev_rigidity_variant.argtypes = [ctypes.c_int]
dev = torch.device("cuda:0")
B = 32
ITERS = int(os.environ.get("RIGID_ITERS", "20"))
for V2 in [int(a) for a in sys.argv[1:]] or [1024, 2048]:
    scenes = [_rigid_scene(V2, 100 + b) for b in range(B)]
    cand = torch.from_numpy(np.stack([s[2] for s in scenes])).to(dev)
    cad = torch.from_numpy(np.stack([s[0] for s in scenes])).to(dev)
    pc = torch.from_numpy(np.stack([s[1] for s in scenes])).to(dev)
    ncand = torch.full((B,), cand.shape[1], dtype=torch.int32, device=dev)
    thr = ops.rigidity_thresholds([s[3] for s in scenes], dev)
    res = {}
    variants = [int(v) for v in os.environ.get("RIGID_VARS", "3,2,0").split(",")]
    for var in variants:
        L.pkdev_rigidity_variant(var)
        for _ in range(3):
            rows, n = ops.rigidity_filter(cand, ncand, cad, pc, thr)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = ITERS
        e0.record()
        for _ in range(it):
            rows, n = ops.rigidity_filter(cand, ncand, cad, pc, thr)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        res[var] = (rows.cpu(), n.cpu())
        nl = cand.shape[1]
        flop = 10.0 * B * nl * nl  # the bench's accounting: ~20 flop per unordered pair of round 1
        print(f"V2={V2} n={nl} variant={var}: {ms * 1e3:8.1f} us per filter (3 rounds), "
              f"{flop / ms / 1e9:6.1f} TFLOP/s = {flop / ms / 1e9 / 157.3:.3f} of f32 VALU; survivors {int(n.sum())}")
    for var in variants:
        same = torch.equal(res[0][1], res[var][1]) and all(
            torch.equal(res[0][0][b, :res[0][1][b]], res[var][0][b, :res[var][1][b]]) for b in range(B))
        print(f"V2={V2}: variant {var} survivors identical to variant 0's: {same}")
    L.pkdev_rigidity_variant(0)
