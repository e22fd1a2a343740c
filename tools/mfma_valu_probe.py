"""MFMA / VALU co-issue probe (pkdev_probe_mfma_valu, csrc/devprobe.hip): 256 blocks x 8 waves,
each wave `iters` tiles of 2 x 8 v_mfma_f32_16x16x4f32 plus NV independent v_min_i32 per 8 MFMAs
(NV per tile-column: top-1 selection ~ 12, a top-2 stream selection ~ 32). Prints us per launch
and cycles per 8 MFMAs at the measured time; flat time vs NV = the VALU hides under the MFMAs."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

from dpfm_amd import _lib  # noqa: E402
_lib.use_dev_lib()

L = _lib.lib()
L.pkdev_probe_mfma_valu.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_void_p]
dev = torch.device("cuda:0")
seed = torch.randn(1024, device=dev)
blocks, iters = 256, 256
out = torch.empty(blocks * 512, device=dev)
st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
for nv in (0, 8, 16, 24, 32, 48, 64):
    f = lambda: L.pkdev_probe_mfma_valu(ctypes.c_void_p(seed.data_ptr()), blocks, iters, nv,  # noqa: E731
                                        ctypes.c_void_p(out.data_ptr()), st())
    for _ in range(100):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    mfma_per_simd = 2 * iters * 16  # 2 waves per SIMD x iters x 16 MFMAs
    tf = blocks * 8 * iters * 16 * 2048 / (us * 1e-6) / 1e12
    print(f"NV={nv:3d} per 8 MFMAs: {us:8.2f} us/launch, {tf:6.1f} TFLOP/s, "
          f"{us * 1e-6 * 2.4e9 / mfma_per_simd * 8:7.1f} cycles@2.4GHz per 8 MFMAs per SIMD", flush=True)
