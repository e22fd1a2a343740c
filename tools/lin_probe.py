"""Memory-stream probes of the per-point layer shapes (pkdev_probe_linear, csrc/devprobe.hip) next
to the production 128 -> 64 rows kernel and a torch copy of the same bytes, at R = 65,536 (the
step's size) and 4x / 16x that (does the rate depend on the launch size?). Graph-replayed."""
import ctypes
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402
from dpfm_amd import _lib, ops  # noqa: E402
_lib.use_dev_lib()  # pkdev_* hooks: libposekern_dev.so (Makefile)

L = _lib.lib()
L.pkdev_probe_linear.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                 ctypes.c_void_p]
L.pkdev_linear_rows_var.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")


def timed(f, n=20):
    f()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                f()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for R in (65536, 262144, 1048576):
    x = torch.randn(R, 128, device=dev)
    w = torch.randn(64, 128, device=dev)
    b = torch.randn(64, device=dev)
    y = torch.empty(R, 64, device=dev)
    byts = 4.0 * R * 192
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    rows = {"layer 128->64 (production)": lambda: L.pkdev_linear_rows_var(x.data_ptr(), w.data_ptr(), b.data_ptr(), R,
                                                                          128, y.data_ptr(), 0, 0, st()),
            "layer no-MFMA": lambda: L.pkdev_linear_rows_var(x.data_ptr(), w.data_ptr(), b.data_ptr(), R, 128,
                                                             y.data_ptr(), 1, 0, st()),
            "layer weight-stationary": lambda: L.pkdev_linear_rows_var(x.data_ptr(), w.data_ptr(), b.data_ptr(), R,
                                                                       128, y.data_ptr(), 5, 1024, st())}
    for mode, name in enumerate(("probe lane-linear", "probe fragment + D stores", "probe + weight staging",
                                 "probe fragment + 16-B stores")):
        rows[name] = (lambda m: lambda: L.pkdev_probe_linear(x.data_ptr(), w.data_ptr(), y.data_ptr(), R, m, st()))(mode)
    xs = x[:, :64]
    rows["torch y.copy_(x[:, :64] + x[:, 64:])"] = lambda: torch.add(x[:, :64], x[:, 64:], out=y)
    for name, f in rows.items():
        us = timed(f)
        print(f"R={R:8d} {name:40s} {us:8.2f} us {byts / us / 1e3:6.0f} GB/s", flush=True)
    del x, y
