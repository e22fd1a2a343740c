"""Rows-kernel limiter study (pkdev_linear_rows_var): production / no-MFMA / no-store /
no-scheduling-barrier variants of y = x W^T + b (Cin 64 | 128 -> 64, R = 65536), over grid
sizes, graph-replayed (50 launches) so host launch gaps are off the clock."""
import ctypes
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402
from dpfm_amd import _lib  # noqa: E402
_lib.use_dev_lib()  # pkdev_* hooks: libposekern_dev.so (Makefile)

L = _lib.lib()
L.pkdev_linear_rows_var.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
R = 65536
names = {0: "production", 1: "no-MFMA", 2: "no-store", 3: "no-sched-barrier", 4: "weight-stat. 2w/SIMD", 5: "weight-stat. 1w/SIMD"}
for cin in (128, 64):
    x = torch.randn(R, cin, device=dev)
    w = torch.randn(64, cin, device=dev)
    b = torch.randn(64, device=dev)
    y = torch.empty(R, 64, device=dev)
    for var in (0, 2, 4, 5):
        for blocks in (0, 256, 512):
            f = lambda: L.pkdev_linear_rows_var(x.data_ptr(), w.data_ptr(), b.data_ptr(), R, cin, y.data_ptr(),  # noqa
                                                var, blocks, torch.cuda.current_stream().cuda_stream)
            assert f() == 0
            torch.cuda.synchronize()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    for _ in range(50):
                        f()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            byts = 4.0 * R * (cin + 64)
            print(f"{cin}->64 {names[var]:17s} blocks={blocks or 'prod':>4}: {us:6.2f} us  {byts / us / 1e3:6.0f} GB/s  "
                  f"{2 * R * cin * 64 / us / 1e6:6.1f} TF/s", flush=True)
