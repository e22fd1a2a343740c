"""Which scalar recipe reproduces v_mfma_f32_16x16x4f32's accumulation bit for bit
(pkdev_probe_mfma_order): H1 one fmaf chain over k in order, H2 per instruction exact products
summed with the accumulator (one rounding), H3 per instruction an fmaf chain onto the accumulator.
Prints the fraction of outputs each recipe matches, on random and on feature-distance-like data."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

from dpfm_amd import _lib  # noqa: E402
_lib.use_dev_lib()
L = _lib.lib()
L.pkdev_probe_mfma_order.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda:0")
T = 4096
g = torch.Generator().manual_seed(0)
for name, A, B in [
        ("randn", torch.randn(T, 16, 32, generator=g), torch.randn(T, 32, 16, generator=g)),
        ("wide-exponent", torch.randn(T, 16, 32, generator=g) * torch.exp(4 * torch.randn(T, 16, 32, generator=g)),
         torch.randn(T, 32, 16, generator=g) * torch.exp(4 * torch.randn(T, 32, 16, generator=g))),
        ("cancelling", torch.randn(T, 16, 32, generator=g).round(decimals=3), torch.randn(T, 32, 16, generator=g))]:
    if name == "cancelling":  # duplicated terms of opposite sign: heavy cancellation inside one instruction
        A[:, :, 1::2] = -A[:, :, 0::2]
        B[:, 1::2, :] = B[:, 0::2, :]
    a, b = A.to(dev).contiguous(), B.to(dev).contiguous()
    out = torch.empty(T, 4, 256, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.pkdev_probe_mfma_order(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), T,
                                    ctypes.c_void_p(out.data_ptr()), st) == 0
    torch.cuda.synchronize()
    o = out.cpu()
    m = o[:, 0].view(torch.int32)
    res = {h: float((o[:, k].view(torch.int32) == m).float().mean()) for k, h in ((1, "H1 fmaf chain"),
                                                                               (2, "H2 exact dot4 + acc"),
                                                                               (3, "H3 fmaf dot4 then + acc"))}
    print(name, res, flush=True)
