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

from typing import Optional

from . import ops

_SIDE = None  # the active GroupedWgrad (TrainStep's backward), or None
FOLD_RELU = True  # fold a producer layer's ReLU backward into the consumer's input gradient
# input gradients whose producer ReLU mask a consumer already applied: (dx storage pointer,
# mask storage pointer) -> dx's version counter when the mask was applied. Keyed by storage, not
# by tensor object: autograd hands the producer a transposed view of the consumer's dx for
# channels-first layers (a new Python object, same storage and version counter). The version
# check rejects a dx that autograd has since accumulated another consumer's gradient into (in
# place, same pointer). The entry holds dx itself, so its memory cannot be handed to another
# tensor while the entry exists (an address match is the same storage), and the producer's
# backward pops it (a stale entry of an earlier backward could otherwise match a new tensor at a
# reused address with the same version 0 and skip a ReLU backward).
_MASKED = {}


def _masked_put(dx, mask) -> None:
    """Record that dx already carries the ReLU mask `mask` (an entry whose producer never runs
    its backward, e.g. one that needs no input gradient, is dropped with the rest past 512)."""
    if len(_MASKED) > 512:
        _MASKED.clear()
    _MASKED[(dx.data_ptr(), mask.data_ptr())] = (dx._version, dx)


def _masked_pop(dy, y) -> bool:
    """True when the consumer of `dy` already applied the ReLU mask `y` (and drops the entry)."""
    if not _MASKED:
        return False
    ent = _MASKED.pop((dy.data_ptr(), y.data_ptr()), None)
    return ent is not None and ent[0] == dy._version


class GroupedWgrad:
    """Weight gradients of all per-point layers of one backward in two launches.

    Each layer's backward records (x, dy) instead of launching pk_linear_wgrad (two
    launches per layer, 56 per training step, each too small to fill the chip) and returns
    None for its weight / bias so autograd leaves their .grad alone. `end()` issues one
    grouped pk_linear_wgrad_grouped on the same stream, writing into persistent .grad
    buffers; a weight used twice in the forward (the refinement layer, modeling/dpfm.py:
    100-104; first/last_lin on both shapes) accumulates in autograd's order. Everything
    stays on one stream: a single-stream HIP graph replays without cross-queue
    dependencies (a forked side stream measured slower on MI355X)."""

    def __init__(self, params, bufs=None, direct_params=()):
        """params: the per-point layers' weights / biases (gradients from the grouped launch);
        direct_params: parameters whose gradient a kernel may write whole through direct() (the
        diffusion times under the fused encoder) and that otherwise get autograd's ordinary
        accumulation (the non-fused encoder path) — never zeroed by end()."""
        self.params = [p for p in params]
        self.direct_params = [p for p in direct_params]
        self.direct_ids = {id(p) for p in self.direct_params}
        self.caller_bufs = bufs is not None
        # persistent .grad buffers (optionally the caller's, e.g. views of one flat buffer the
        # caller zeroes before each backward)
        self.bufs = {id(p): (bufs[id(p)] if bufs is not None else
                             torch.zeros_like(p, memory_format=torch.contiguous_format))
                     for p in self.params + self.direct_params}
        self.seen = set()
        self.calls = []

    def begin(self):
        global _SIDE
        _MASKED.clear()
        for p in self.params:
            p.grad = self.bufs[id(p)]
        for p in self.direct_params:
            # autograd accumulates into .grad when no kernel writes it whole: start it from zero
            # (a caller's flat buffer is already zeroed; an own buffer holds the last step's value)
            if not self.caller_bufs:
                self.bufs[id(p)].zero_()
            p.grad = self.bufs[id(p)]
        self.seen = set()
        self.calls = []
        _SIDE = self

    def owns(self, p) -> bool:
        return id(p) in self.bufs

    def direct(self, p):
        """p's persistent .grad buffer for a kernel that writes p's whole gradient itself (e.g. the
        diffusion-time gradient of pk_spectral_diffusion's backward), on p's first use in this
        backward; None otherwise (the caller then returns the gradient to autograd)."""
        if id(p) not in self.bufs or id(p) in self.seen:
            return None
        self.seen.add(id(p))
        return self.bufs[id(p)]

    def launch(self, x, dy, weight, bias, channels_first: bool):
        acc = id(weight) in self.seen
        self.seen.add(id(weight))
        if bias is not None:
            self.seen.add(id(bias))
        dw = self.bufs[id(weight)]
        db = self.bufs[id(bias)] if bias is not None else None
        self.calls.append((x, dy, channels_first, dw.view(dw.shape[0], -1), db, acc))

    @staticmethod
    def _groupable(c) -> bool:
        x, dy, cf, dw, _, _ = c
        O, I = dw.shape
        return ((O + 31) // 32) * ((I + 31) // 32) <= 8

    def end(self, run: bool = True):
        global _SIDE
        _SIDE = None
        if run:
            if all(self._groupable(c) for c in self.calls):
                ops.linear_wgrad_grouped(self.calls)
            else:  # a shape outside the grouped kernel's range: one launch pair per call, in order
                for x, dy, cf, dw, db, acc in self.calls:
                    ops.linear_wgrad(x, dy, channels_first=cf, want_bias=db is not None, dw=dw, db=db,
                                     accumulate=acc)
            for p in self.params:  # a layer the forward did not use gets a zero gradient
                if id(p) not in self.seen:
                    p.grad.zero_()
            # (direct_params: written by direct(), or accumulated by autograd into the zeroed buffer)
        self.calls = []


def _side_owns(weight, bias) -> bool:
    return _SIDE is not None and _SIDE.owns(weight) and (bias is None or _SIDE.owns(bias))


class _PointwiseFn(torch.autograd.Function):
    """y = x W^T (+ b) over every point of x in its NATIVE layout: cf=False rows [..., C],
    cf=True channels-first [B, C, N]. The modules below pick the native layout from the
    input's strides (a transposed view of a contiguous tensor runs on that tensor), so the
    reference's transposes (modeling/dpfm.py:90-91, 113-116) cost no copies."""

    @staticmethod
    def forward(ctx, x, weight, bias, cf, relu, in_relu, sigmoid=False):
        w2 = weight.view(weight.shape[0], -1)
        ctx.has_bias, ctx.cf, ctx.relu, ctx.sigmoid = bias is not None, cf, relu, sigmoid
        ctx.param, ctx.bias = weight, bias  # the Parameter objects (GroupedWgrad's buffer keys)
        # a fresh (non-view) output: the reference applies in-place ReLUs to it (:112-116);
        # relu=True applies the following nn.ReLU in the kernel's epilogue instead, sigmoid=True
        # the following nn.Sigmoid (the overlap head's last layer, modeling/dpfm.py:132-137)
        if sigmoid:
            Cout, Cin = w2.shape
            if cf:
                Bn, _, N = x.shape
                y = torch.empty((Bn, Cout, N), dtype=x.dtype, device=x.device)
                ops.linear_ex(x, w2, bias, 1, Bn * N, N, Cin, Cout, y=y, act=2)
            else:
                y = torch.empty(x.shape[:-1] + (Cout,), dtype=x.dtype, device=x.device)
                ops.linear_ex(x, w2, bias, 0, x.numel() // Cin, 0, Cin, Cout, y=y, act=2)
        else:
            y = ops.linear_fwd(x, w2, bias, channels_first=cf, relu=relu)
        # this layer's input gradient can apply the ReLU backward of the layer that produced x
        ctx.in_relu = FOLD_RELU and in_relu
        ctx.save_for_backward(x, weight, y if (relu or sigmoid) else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        w2 = weight.view(weight.shape[0], -1)
        cf = ctx.cf
        dy = dy.contiguous()
        if ctx.relu and not _masked_pop(dy, y):
            # the fused ReLU's backward (aten's ReluBackward: threshold_backward on the output),
            # unless the consuming layer already applied it in its input-gradient epilogue
            dy = torch.ops.aten.threshold_backward(dy, y, 0.0)
        dx = dw = db = None
        if ctx.sigmoid:
            # the sigmoid's backward dy y (1 - y) folded into the input gradient's prologue, the
            # scaled dy written out for the weight gradient (pk_linear_ex pre / pre_out)
            Cout, Cin = w2.shape
            dz = torch.empty_like(dy)
            dx = torch.empty_like(x)
            if cf:
                Bn, _, N = x.shape
                ops.linear_ex(dy, w2, None, 1, Bn * N, N, Cout, Cin, y=dx, transw=True,
                              mask=x if ctx.in_relu else None, pre=y, pre_out=dz)
            else:
                ops.linear_ex(dy, w2, None, 0, dy.numel() // Cout, 0, Cout, Cin, y=dx, transw=True,
                              mask=x if ctx.in_relu else None, pre=y, pre_out=dz)
            if ctx.in_relu:
                _masked_put(dx, x)
            dy = dz
        elif ctx.needs_input_grad[0]:
            # dy W (rows) / W^T dy (cf); with in_relu the producer's ReLU backward is folded in
            dx = ops.linear_fwd(dy, w2, None, channels_first=cf, transw=True, mask=x if ctx.in_relu else None)
            if ctx.in_relu:
                _masked_put(dx, x)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            if _side_owns(ctx.param, ctx.bias):
                _SIDE.launch(x, dy, ctx.param, ctx.bias, channels_first=cf)
            else:
                dw, db = ops.linear_wgrad(x, dy, channels_first=cf, want_bias=ctx.has_bias)
                dw = dw.view(weight.shape)
        return dx, dw, db, None, None, None, None


class _PointwiseResidualFn(torch.autograd.Function):
    """y = W x + b + res for a channels-first [B, C, N] layer (the residual add of
    modeling/dpfm.py:101-103, desc = desc + layer(...), folded into the layer's epilogue:
    pk_linear_ex `add`). Backward: dres = dy, the input gradient and the grouped weight
    gradients as _PointwiseFn's."""

    @staticmethod
    def forward(ctx, x, weight, bias, res, in_relu):
        w2 = weight.view(weight.shape[0], -1)
        Cout, Cin = w2.shape
        Bn, _, N = x.shape
        y = torch.empty((Bn, Cout, N), dtype=x.dtype, device=x.device)
        ops.linear_ex(x, w2, bias, 1, Bn * N, N, Cin, Cout, y=y, add=res, add_cols=Cout)
        ctx.param, ctx.bias, ctx.has_bias = weight, bias, bias is not None
        ctx.in_relu = FOLD_RELU and in_relu
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        w2 = weight.view(weight.shape[0], -1)
        dy = dy.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = ops.linear_fwd(dy, w2, None, channels_first=True, transw=True, mask=x if ctx.in_relu else None)
            if ctx.in_relu:
                _masked_put(dx, x)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            if _side_owns(ctx.param, ctx.bias):
                _SIDE.launch(x, dy, ctx.param, ctx.bias, channels_first=True)
            else:
                dw, db = ops.linear_wgrad(x, dy, channels_first=True, want_bias=ctx.has_bias)
                dw = dw.view(weight.shape)
        return dx, dw, db, dy if ctx.needs_input_grad[3] else None, None


class _LinearPairCfFn(torch.autograd.Function):
    """The refinement's first_lin on both shapes at once (modeling/dpfm.py:98, desc =
    first_lin(x).transpose(1, 2) for x = features_x, features_y) from the encoder's concatenated
    rows-layout features [2B, N, Cin]: one launch writing channels-first [2B, Cout, N]
    (pk_linear_ex store_cf), returned as the two shapes' desc [B0, Cout, N] and [2B - B0, Cout, N]
    — no transpose copies and no concatenation of the two features' gradients. Backward: the two
    channels-first gradients into one rows-layout dy (pk_transpose_cf_rows), the features'
    gradient in one launch, the weight gradient recorded once for both shapes."""

    @staticmethod
    def forward(ctx, feat, weight, bias, B0):
        B2, N, Cin = feat.shape
        w2 = weight.view(weight.shape[0], -1)
        Cout = w2.shape[0]
        y = torch.empty((B2, Cout, N), dtype=feat.dtype, device=feat.device)
        ops.linear_ex(feat, w2, bias, 0, B2 * N, N, Cin, Cout, y=y, store_cf=True)
        ctx.B0, ctx.param, ctx.bias, ctx.has_bias = B0, weight, bias, bias is not None
        ctx.save_for_backward(feat, weight)
        return y[:B0], y[B0:]

    @staticmethod
    def backward(ctx, g0, g1):
        feat, weight = ctx.saved_tensors
        w2 = weight.view(weight.shape[0], -1)
        B2, N, Cin = feat.shape
        Cout = w2.shape[0]
        g0, g1 = g0.contiguous(), g1.contiguous()
        dyr = torch.empty((B2, N, Cout), dtype=feat.dtype, device=feat.device)
        ops._lib.call("pk_transpose_cf_rows", ops._lib.ptr(g0), ops._lib.ptr(g1), ctx.B0, B2, Cout, N, Cout * N,
                      ops._lib.ptr(dyr), ops._lib.stream(feat.device), work=("hbm", 8 * B2 * N * Cout))
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = ops.linear_fwd(dyr, w2, None, channels_first=False, transw=True)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            if _side_owns(ctx.param, ctx.bias):
                _SIDE.launch(feat, dyr, ctx.param, ctx.bias, channels_first=False)
            else:
                dw, db = ops.linear_wgrad(feat, dyr, channels_first=False, want_bias=ctx.has_bias)
                dw = dw.view(weight.shape)
        return dx, dw, db, None


def linear_pair_cf(layer: "Linear", feat: torch.Tensor, B0: int):
    """(desc0, desc1) = layer(feat[:B0]).transpose(1, 2), layer(feat[B0:]).transpose(1, 2) as two
    contiguous channels-first tensors (_LinearPairCfFn), or None outside its shapes."""
    Cin, Cout = layer.in_features, layer.out_features
    if not (feat.is_cuda and feat.dim() == 3 and feat.is_contiguous() and feat.dtype == torch.float32
            and feat.shape[-1] == Cin and 0 < B0 < feat.shape[0] and Cin in (16, 32, 64, 128)
            and Cout in (16, 32, 64, 128) and not layer.relu_out and not layer.sigmoid_out):
        # (Cout: the widths the backward's pk_transpose_cf_rows instantiates)
        return None
    return _LinearPairCfFn.apply(feat, layer.weight, layer.bias, B0)


def pointwise_residual(layer: "Conv1d", x: torch.Tensor, res: torch.Tensor) -> torch.Tensor:
    """res + layer(x) for a Conv1d(k=1) layer on channels-first [B, C, N] tensors in one launch
    (falls back to the two-step form for other storage orders)."""
    if (x.is_cuda and x.dim() == 3 and x.is_contiguous() and res.is_contiguous() and res.shape[1] == layer.out_channels
            and res.shape[0] == x.shape[0] and res.shape[2] == x.shape[2] and res.dtype == x.dtype
            and layer.in_channels in (16, 32, 64, 128)):  # the cf MFMA kernel's range
        return _PointwiseResidualFn.apply(x, layer.weight, layer.bias, res, getattr(x, "_pk_relu_out", False))
    return res + layer(x)


def _pointwise(x, weight, bias, sem_cf: bool, out_cf: Optional[bool] = None, relu: bool = False,
               sigmoid: bool = False):
    """Apply the layer to x of semantic layout sem_cf (False: [..., C]; True: [B, C, N]).
    out_cf: force the output storage layout (None: the native layout of the input)."""
    if not x.is_cuda:
        raise ops._lib.PoseKernError("dpfm_amd layers run on HIP devices only (no CPU fallback)")
    if x.dim() == 3 and not x.is_contiguous() and x.transpose(1, 2).is_contiguous():
        base, native_cf = x.transpose(1, 2), not sem_cf
    else:
        base, native_cf = x.contiguous(), sem_cf
    in_relu = getattr(x, "_pk_relu_out", False)
    y = _PointwiseFn.apply(base, weight, bias, native_cf, relu, in_relu, sigmoid)
    if out_cf is not None and out_cf != native_cf and y.dim() == 3:
        y = y.transpose(1, 2).contiguous().transpose(1, 2)  # same values, other storage order
    out = y if native_cf == sem_cf else y.transpose(1, 2)
    if relu:  # marks the tensor the consumer sees (a view object when the layout flips)
        out._pk_relu_out = True
    return out


class Linear(nn.Linear):
    """nn.Linear over every point; `out_cf = True` stores the [B, N, C] output
    channels-first (a transposed view of a [B, C, N] tensor) for a channels-first consumer;
    `relu_out = True` applies the ReLU that follows the layer in the reference (the module
    holding that ReLU is then an nn.Identity, so state_dict keys are unchanged)."""
    out_cf: Optional[bool] = None
    relu_out: bool = False
    sigmoid_out: bool = False  # the following nn.Sigmoid in the epilogue (thin layers, Cout <= 4)

    def forward(self, x):
        sig = self.sigmoid_out and (self.out_features <= 4 or self.in_features <= 4)
        y = _pointwise(x, self.weight, self.bias, sem_cf=False, out_cf=self.out_cf, relu=self.relu_out, sigmoid=sig)
        return torch.sigmoid(y) if (self.sigmoid_out and not sig) else y


class Conv1d(nn.Conv1d):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.kernel_size != (1,) or self.stride != (1,) or self.padding != (0,) or self.groups != 1:
            raise ValueError("only the reference's pointwise Conv1d(kernel_size=1) is supported")

    def forward(self, x):
        return _pointwise(x, self.weight, self.bias, sem_cf=True)
