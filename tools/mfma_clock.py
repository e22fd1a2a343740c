"""MFMA clock probe (pkdev_probe_mfma, csrc/devprobe.hip): 512 blocks x 8 waves, each wave
`iters` x 4 chains x 8 v_mfma_f32_16x16x4f32 (the feature-distance pass's per-tile shape and
its per-SIMD MFMA count at iters = 8), graph-replayed; prints us per launch, the implied
TFLOP/s and the in-kernel clock from s_memtime / s_memrealtime (100 MHz)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

from dpfm_amd import _lib  # noqa: E402
_lib.use_dev_lib()  # pkdev_* hooks: libposekern_dev.so (Makefile)

L = _lib.lib()
L.pkdev_probe_mfma.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
dev = torch.device("cuda:0")
seed = torch.randn(1024, device=dev)
blocks = 512
out = torch.empty(blocks * 512, device=dev)
stamp = torch.zeros(4, dtype=torch.int64, device=dev)
st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
for iters in (8, 64, 512):
    f = lambda: L.pkdev_probe_mfma(ctypes.c_void_p(seed.data_ptr()), blocks, iters,  # noqa: E731
                                   ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stamp.data_ptr()), st())
    for _ in range(200):  # warm the clock
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 100
    n_mfma = blocks * 8 * iters * 4 * 8
    fl = n_mfma * 2048
    t = stamp.cpu().tolist()
    clk = (t[1] - t[0]) / max(t[3] - t[2], 1) * 100  # MHz
    cyc_per_simd = n_mfma * 32 / 1024
    print(f"iters={iters}: {us:.1f} us/launch, {fl / us / 1e6:.1f} TFLOP/s = {fl / us / 1e6 / 157.3:.3f} of 157.3; "
          f"in-kernel clock {clk:.0f} MHz; MFMA cycles per SIMD {cyc_per_simd:.0f} = {cyc_per_simd / clk:.1f} us at that clock",
          flush=True)
