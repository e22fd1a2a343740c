"""Per-point layers of the model path with their weight gradients in HIP.

`Linear` and `Conv1d` are drop-in subclasses of torch.nn.Linear / Conv1d(kernel_size=1):
same constructor, parameter names and state_dict keys (weights/weights.pt loads
unchanged). All three products run in HIP on the f32 MFMA: the forward (bias fused) and
the input gradient in pk_linear_fwd (32 points x all outputs per wave, weight in LDS,
either layout, so no transposes or bias kernels), the weight / bias gradients — a
reduction over all B*N points into a <= 128 x 128 matrix — in pk_linear_wgrad, which
splits the points across the whole chip.
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
        # a fresh (non-view) output: the reference applies in-place ReLUs to it (:112-116)
        return ops.linear_fwd(x, weight, bias, channels_first=False)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = ops.linear_fwd(dy, weight, None, channels_first=False, transw=True)  # dy W
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw, db = ops.linear_wgrad(x, dy, channels_first=False, want_bias=ctx.has_bias)
        return dx, dw, db


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        # y[b] = W x[b] (+ b) over every point, bias fused (no MIOpen convolution)
        return ops.linear_fwd(x, weight[:, :, 0], bias, channels_first=True)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = ops.linear_fwd(dy, weight[:, :, 0], None, channels_first=True, transw=True)  # W^T dy
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
