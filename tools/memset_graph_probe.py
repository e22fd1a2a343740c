"""Dev probe: are memset / memcpy nodes of a captured HIP graph ordered against the
kernels around them on replay? Each case writes a buffer with a slow kernel, then a
memset / D2D memcpy node, then a reader kernel; replayed many times, checked each time.

  python tools/memset_graph_probe.py
"""
import ctypes
import os
import sys

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
n = 1 << 20
A = torch.randn(2048, 2048, device=dev)


def slow_write(x, v):
    # a few ms of work whose result lands in x (x = v exactly)
    t = A @ A
    t = t @ A
    x.copy_((t[: x.numel() // 2048 + 1].reshape(-1)[: x.numel()] * 0 + v).view_as(x))


def case_memset():
    x = torch.empty(n, dtype=torch.float32, device=dev)
    y = torch.empty_like(x)

    def body():
        s = torch.cuda.current_stream().cuda_stream  # the capture stream while capturing
        slow_write(x, 7.0)
        assert hip.hipMemsetAsync(x.data_ptr(), 0, x.numel() * 4, s) == 0
        y.copy_(x * 1.0)
    return body, lambda: bool((y == 0).all())


def case_memcpy():
    x = torch.empty(n, dtype=torch.float32, device=dev)
    z = torch.empty_like(x)
    y = torch.empty_like(x)

    def body():
        s = torch.cuda.current_stream().cuda_stream  # the capture stream while capturing
        slow_write(x, 5.0)
        assert hip.hipMemcpyAsync(z.data_ptr(), x.data_ptr(), x.numel() * 4, 3, s) == 0
        y.copy_(z * 1.0)
        slow_write(x, 9.0)  # must not leak into this replay's z
    return body, lambda: bool((y == 5).all())


def case_memset_first():
    x = torch.empty(n, dtype=torch.float32, device=dev)

    def body():
        s = torch.cuda.current_stream().cuda_stream  # the capture stream while capturing
        assert hip.hipMemsetAsync(x.data_ptr(), 0, x.numel() * 4, s) == 0
        x.add_(1.0)
    return body, lambda: bool((x == 1).all())


for name, case in (("memset-after-kernel", case_memset), ("memcpy-between-kernels", case_memcpy),
                   ("memset-first-node", case_memset_first)):
    body, check = case()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    bad_sync = bad_back = 0
    for r in range(20):
        g.replay()
        torch.cuda.synchronize()
        bad_sync += 0 if check() else 1
    for r in range(20):  # back-to-back replays, one check at the end
        g.replay()
    torch.cuda.synchronize()
    bad_back = 0 if check() else 1
    print(f"{name}: wrong after {bad_sync}/20 synced replays; back-to-back final {'WRONG' if bad_back else 'ok'}",
          flush=True)
print("done")
