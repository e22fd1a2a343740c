"""Per-point layers of the model path with their weight gradients in HIP.

`Linear` and `Conv1d` are drop-in subclasses of torch.nn.Linear / Conv1d(kernel_size=1):
same constructor, parameter names and state_dict keys (weights/weights.pt loads
unchanged). Forward and input-gradient products are large-M GEMMs (hipBLASLt); the
weight / bias gradients — a reduction over all B*N points into a <= 128 x 128 matrix,
which a library GEMM runs on a handful of output tiles — go to pk_linear_wgrad, which
splits the points across the whole chip (ops.linear_wgrad).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        O, I = weight.shape
        # a fresh (non-view) output: the reference applies in-place ReLUs to it (:112-116)
        y = torch.empty(x.shape[:-1] + (O,), dtype=x.dtype, device=x.device)
        x2, y2 = x.reshape(-1, I), y.view(-1, O)
        if bias is not None:
            torch.addmm(bias, x2, weight.t(), out=y2)
        else:
            torch.mm(x2, weight.t(), out=y2)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.matmul(dy, weight)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw, db = ops.linear_wgrad(x, dy, channels_first=False, want_bias=ctx.has_bias)
        return dx, dw, db


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        # y[b] = W x[b] (+ b): a batched GEMM (no MIOpen convolution on the path)
        y = torch.bmm(weight[:, :, 0].expand(x.shape[0], -1, -1), x)
        if bias is not None:
            y.add_(bias[:, None])
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.matmul(weight[:, :, 0].t(), dy)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw, db = ops.linear_wgrad(x, dy, channels_first=True, want_bias=ctx.has_bias)
            dw = dw[:, :, None]
        return dx, dw, db


class Linear(nn.Linear):
    def forward(self, x):
        if not x.is_cuda:
            raise ops._lib.PoseKernError("dpfm_amd layers run on HIP devices only (no CPU fallback)")
        return _LinearFn.apply(x, self.weight, self.bias)


class Conv1d(nn.Conv1d):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.kernel_size != (1,) or self.stride != (1,) or self.padding != (0,) or self.groups != 1:
            raise ValueError("only the reference's pointwise Conv1d(kernel_size=1) is supported")

    def forward(self, x):
        if not x.is_cuda:
            raise ops._lib.PoseKernError("dpfm_amd layers run on HIP devices only (no CPU fallback)")
        return _Conv1x1Fn.apply(x, self.weight, self.bias)
