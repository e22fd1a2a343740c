"""Spectral DiffusionNet encoder — the DPFM point encoder (H7).

Mirrors upstream diffusion-net `layers.py` as vendored by the DPFM submodule (imported at
models/dpfm.py:11, built at models/dpfm.py:22-30 with C_in=3, C_out=32, C_width=64,
N_block=2, dropout=False, with_gradient_features=False): same module and parameter
names as weights/weights.pt (`first_lin`, `block_{i}.diffusion.diffusion_time`,
`block_{i}.mlp.miniMLP_mlp_layer_{000,001,002}`, `last_lin`).

The diffusion step (to_basis -> exp(-lambda t) -> from_basis) runs in one fused HIP kernel
per direction (ops.spectral_diffusion); the per-point MLPs are GEMMs.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from .layers import Linear

# The whole configured DiffusionNet as one autograd node (_EncoderFn); False runs the per-module
# path (the parity tests compare the two)
FUSED_ENCODER = True


class LearnedTimeDiffusion(nn.Module):
    def __init__(self, C_inout: int, method: str = "spectral"):
        super().__init__()
        if method != "spectral":
            raise ValueError("only spectral diffusion is on the hot path (models/dpfm.py:22-30)")
        self.C_inout = C_inout
        self.diffusion_time = nn.Parameter(torch.zeros(C_inout))

    def forward(self, x, L, mass, evals, evecs):
        # upstream clamps diffusion_time in place (clamp_(min=1e-8)) before
        # every diffusion; the spectral kernel applies and writes back that clamp itself (same
        # storage, so HIP-graph replays see it), saving a launch per block
        return ops.spectral_diffusion(x, mass, evals, evecs, self.diffusion_time, clamp_t=True)


class MiniMLP(nn.Sequential):
    def __init__(self, layer_sizes, dropout=False, activation=nn.ReLU, name="miniMLP"):
        super().__init__()
        for i in range(len(layer_sizes) - 1):
            if dropout and i > 0:
                self.add_module(name + "_mlp_layer_dropout_{:03d}".format(i), nn.Dropout(p=0.5))
            lin = Linear(layer_sizes[i], layer_sizes[i + 1])
            self.add_module(name + "_mlp_layer_{:03d}".format(i), lin)
            if i + 2 != len(layer_sizes):
                if activation is nn.ReLU:  # fused into the layer's epilogue (same module names)
                    lin.relu_out = True
                    self.add_module(name + "_mlp_act_{:03d}".format(i), nn.Identity())
                else:
                    self.add_module(name + "_mlp_act_{:03d}".format(i), activation())


class _BlockMLPFn(torch.autograd.Function):
    """mlp(cat[x_in, x_diffuse]) + x_in for the configured MiniMLP (128 -> 64 -> 64 -> 64, ReLU
    between): forward in one fused launch (ops.mlp3_fwd); backward through the per-layer
    input-gradient kernels, the ReLU masks on the saved h1 / h2, and the weight gradients
    recorded for the grouped launch (layers.GroupedWgrad) or computed per layer."""

    @staticmethod
    def forward(ctx, x_in, x_diff, w1, b1, w2, b2, w3, b3):
        cat, h1, h2, y = ops.mlp3_fwd(x_in, x_diff, w1, b1, w2, b2, w3, b3)
        ctx.save_for_backward(cat, h1, h2, w1, w2, w3)
        ctx.params = (w1, b1, w2, b2, w3, b3)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import layers
        cat, h1, h2, w1, w2, w3 = ctx.saved_tensors
        P = ctx.params
        dy = dy.contiguous()
        grads = [None] * 6

        def wgrad(x, d, k):  # layer k (0..2): weight P[2k], bias P[2k + 1]
            if layers._side_owns(P[2 * k], P[2 * k + 1]):
                layers._SIDE.launch(x, d, P[2 * k], P[2 * k + 1], channels_first=False)
            else:
                grads[2 * k], grads[2 * k + 1] = ops.linear_wgrad(x, d, channels_first=False, want_bias=True)

        wgrad(h2, dy, 2)
        d2 = torch.ops.aten.threshold_backward(ops.linear_fwd(dy, w3, None, channels_first=False, transw=True), h2, 0.0)
        wgrad(h1, d2, 1)
        d1 = torch.ops.aten.threshold_backward(ops.linear_fwd(d2, w2, None, channels_first=False, transw=True), h1, 0.0)
        wgrad(cat, d1, 0)
        dcat = ops.linear_fwd(d1, w1, None, channels_first=False, transw=True)
        C = dy.shape[-1]
        dx_in = dcat[..., :C] + dy  # the residual
        dx_diff = dcat[..., C:].contiguous()
        return (dx_in, dx_diff, *grads)


class DiffusionNetBlock(nn.Module):
    def __init__(self, C_width, mlp_hidden_dims, dropout=False, diffusion_method="spectral",
                 with_gradient_features=False, with_gradient_rotations=True):
        super().__init__()
        if with_gradient_features:
            raise ValueError("gradient features are off in the reference config (models/dpfm.py:28)")
        self.C_width = C_width
        self.diffusion = LearnedTimeDiffusion(C_width, method=diffusion_method)
        self.mlp = MiniMLP([2 * C_width] + list(mlp_hidden_dims) + [C_width], dropout=dropout)

    # The fused block forward (pk_mlp3_fwd) is opt-in: on MI355X it measured no faster than the
    # per-layer kernels it replaces (46 us vs 20 + 12 + 12 us of layer launches plus the concat
    # and the residual add: one 8-wave block per CU, 103 KB of LDS), DESIGN.md §3
    fused_mlp = False

    def _fusable(self, x_in) -> bool:
        lins = [m for m in self.mlp if isinstance(m, Linear)]
        return (self.fused_mlp and x_in.is_cuda and len(lins) == 3 and self.C_width == 64 and len(self.mlp) == 5
                and all(l.relu_out for l in lins[:2]) and not lins[2].relu_out
                and all(l.bias is not None for l in lins)
                and [tuple(l.weight.shape) for l in lins] == [(64, 128), (64, 64), (64, 64)])

    def forward(self, x_in, mass, L, evals, evecs, gradX, gradY):
        x_diffuse = self.diffusion(x_in, L, mass, evals, evecs)
        if self._fusable(x_in):  # the configured block: one fused forward launch
            l0, l1, l2 = [m for m in self.mlp if isinstance(m, Linear)]
            return _BlockMLPFn.apply(x_in, x_diffuse, l0.weight, l0.bias, l1.weight, l1.bias, l2.weight, l2.bias)
        return self.mlp(torch.cat((x_in, x_diffuse), dim=-1)) + x_in


def _wgrad(x, dy, weight, bias):
    """Weight / bias gradients of a rows-layout layer: recorded for the grouped launch of the
    training step (layers.GroupedWgrad) or computed now. Returns (dw, db) or (None, None)."""
    from . import layers
    if layers._side_owns(weight, bias):
        layers._SIDE.launch(x, dy, weight, bias, channels_first=False)
        return None, None
    dw, db = ops.linear_wgrad(x, dy, channels_first=False, want_bias=bias is not None)
    return dw.view(weight.shape), db


class _EncoderFn(torch.autograd.Function):
    """The configured DiffusionNet (first_lin 3 -> 64, N_block blocks of spectral diffusion +
    MLP 128 -> 64 -> 64 -> 64 with ReLUs and the residual, last_lin 64 -> C_out) over rows
    [R, C] as one autograd node with a hand-written backward, so no concatenation, residual
    add, slice copy or gradient accumulation runs as a separate launch:
      forward : block i works in one [R, 128] buffer CAT_i: x_in in columns 0..63 (written
                there by its producer: first_lin or block i-1's last layer, whose residual add
                is its epilogue), the diffusion writes x_diffuse into columns 64..127;
      backward: the first MLP layer's input gradient is split in its epilogue into dX (columns
                0..63, plus the residual's dy) and dD (64..127); the diffusion backward of dD
                accumulates into dX, which is the previous layer's output gradient.
    Same arithmetic per layer as the module path (models/dpfm.py:22-30; upstream layers.py)."""

    @staticmethod
    def forward(ctx, fcat, mass, evals, evecs, nblock, *params):
        R = fcat.shape[0] * fcat.shape[1]
        B, N = fcat.shape[0], fcat.shape[1]
        dev = fcat.device
        w0, b0 = params[0], params[1]
        wl, bl = params[-2], params[-1]
        blocks = [params[2 + 7 * i: 9 + 7 * i] for i in range(nblock)]
        Cout = wl.shape[0]
        cats = [torch.empty((B, N, 128), dtype=torch.float32, device=dev) for _ in range(nblock)]
        ops.linear_ex(fcat, w0, b0, 0, R, 0, fcat.shape[-1], 64, y=cats[0], ldy=128)
        h1s, h2s, raws = [], [], []
        Y = torch.empty((B, N, 64), dtype=torch.float32, device=dev)
        for i, (t, w1, b1, w2, b2, w3, b3) in enumerate(blocks):
            cat = cats[i]
            raws.append(ops.spectral_raw(cat, 128, mass, evals, evecs, t, True, 0, cat[..., 64:], 128))
            h1 = torch.empty((B, N, 64), dtype=torch.float32, device=dev)
            h2 = torch.empty_like(h1)
            ops.linear_ex(cat, w1, b1, 0, R, 0, 128, 64, y=h1, relu=True)
            ops.linear_ex(h1, w2, b2, 0, R, 0, 64, 64, y=h2, relu=True)
            nxt = cats[i + 1] if i + 1 < nblock else Y
            ops.linear_ex(h2, w3, b3, 0, R, 0, 64, 64, y=nxt, ldy=128 if i + 1 < nblock else 0, add=cat, lda=128,
                          add_cols=64)
            h1s.append(h1)
            h2s.append(h2)
        feat = torch.empty((B, N, Cout), dtype=torch.float32, device=dev)
        ops.linear_ex(Y, wl, bl, 0, R, 0, 64, Cout, y=feat)
        ctx.nblock = nblock
        ctx.save_for_backward(fcat, mass, evals, evecs, Y, *cats, *h1s, *h2s, *raws, *params)
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        nb = ctx.nblock
        sv = ctx.saved_tensors
        fcat, mass, evals, evecs, Y = sv[:5]
        cats = sv[5:5 + nb]
        h1s = sv[5 + nb:5 + 2 * nb]
        h2s = sv[5 + 2 * nb:5 + 3 * nb]
        raws = sv[5 + 3 * nb:5 + 4 * nb]
        params = sv[5 + 4 * nb:]
        w0, b0, wl, bl = params[0], params[1], params[-2], params[-1]
        blocks = [params[2 + 7 * i: 9 + 7 * i] for i in range(nb)]
        B, N = fcat.shape[0], fcat.shape[1]
        R = B * N
        dev = fcat.device
        dfeat = dfeat.contiguous()
        Cout = wl.shape[0]
        grads = [None] * len(params)
        gw = _wgrad(Y, dfeat, wl, bl)
        grads[-2], grads[-1] = gw
        dy = torch.empty((B, N, 64), dtype=torch.float32, device=dev)
        ops.linear_ex(dfeat, wl, None, 0, R, 0, Cout, 64, y=dy, transw=True)
        for i in reversed(range(nb)):
            t, w1, b1, w2, b2, w3, b3 = blocks[i]
            k = 2 + 7 * i
            grads[k + 5], grads[k + 6] = _wgrad(h2s[i], dy, w3, b3)
            d2 = torch.empty_like(dy)
            ops.linear_ex(dy, w3, None, 0, R, 0, 64, 64, y=d2, transw=True, mask=h2s[i])
            grads[k + 3], grads[k + 4] = _wgrad(h1s[i], d2, w2, b2)
            d1 = torch.empty_like(dy)
            ops.linear_ex(d2, w2, None, 0, R, 0, 64, 64, y=d1, transw=True, mask=h1s[i])
            grads[k + 1], grads[k + 2] = _wgrad(cats[i], d1, w1, b1)
            dX = torch.empty_like(dy)
            dD = torch.empty_like(dy)
            # dcat = d1 W1: columns 0..63 (+ the residual's dy) -> dX, 64..127 -> dD
            ops.linear_ex(d1, w1, None, 0, R, 0, 64, 128, y=dX, transw=True, y2=dD, split=64, add=dy, add_cols=64)
            # dL/dt straight into t's persistent .grad when the grouped weight gradient owns it (no
            # autograd accumulation launch)
            from . import layers
            gbuf = layers._SIDE.direct(t) if layers._SIDE is not None else None
            gt = gbuf if gbuf is not None else torch.empty((64,), dtype=torch.float32, device=dev)
            ops.spectral_raw(dD, 64, mass, evals, evecs, t, True, 1, dX, 64, saved=raws[i], gt=gt, accumulate=True)
            grads[k] = None if gbuf is not None else gt
            dy = dX
        grads[0], grads[1] = _wgrad(fcat, dy, w0, b0)
        dfcat = None
        if ctx.needs_input_grad[0]:  # the features are data in DPFM; kept for API completeness
            dfcat = torch.empty_like(fcat)
            ops.linear_ex(dy, w0, None, 0, R, 0, 64, fcat.shape[-1], y=dfcat, transw=True)
        return (dfcat, None, None, None, None, *grads)


class DiffusionNet(nn.Module):
    def __init__(self, C_in, C_out, C_width=128, N_block=4, last_activation=None, outputs_at="vertices",
                 mlp_hidden_dims=None, dropout=True, with_gradient_features=True, with_gradient_rotations=True,
                 diffusion_method="spectral"):
        super().__init__()
        if outputs_at != "vertices":
            raise ValueError("DPFM reads features at vertices")
        self.C_in, self.C_out, self.C_width, self.N_block = C_in, C_out, C_width, N_block
        self.last_activation = last_activation
        if mlp_hidden_dims is None:
            mlp_hidden_dims = [C_width, C_width]
        self.first_lin = Linear(C_in, C_width)
        self.last_lin = Linear(C_width, C_out)
        self.blocks = []
        for i_block in range(N_block):
            blk = DiffusionNetBlock(C_width, mlp_hidden_dims, dropout=dropout, diffusion_method=diffusion_method,
                                    with_gradient_features=with_gradient_features,
                                    with_gradient_rotations=with_gradient_rotations)
            self.blocks.append(blk)
            self.add_module("block_" + str(i_block), blk)

    def _fused_params(self, x_in):
        """The parameter list of _EncoderFn when this is the configured network, else None."""
        if not (x_in.is_cuda and x_in.dtype == torch.float32 and self.C_width == 64 and self.last_activation is None
                and self.first_lin.in_features <= 4 and self.last_lin.out_features in (16, 32, 64)):
            return None
        ps = [self.first_lin.weight, self.first_lin.bias]
        for b in self.blocks:
            lins = [m for m in b.mlp if isinstance(m, Linear)]
            if (len(b.mlp) != 5 or len(lins) != 3 or [tuple(l.weight.shape) for l in lins] != [(64, 128), (64, 64), (64, 64)]
                    or not (lins[0].relu_out and lins[1].relu_out and not lins[2].relu_out)
                    or any(l.bias is None for l in lins) or b.diffusion.diffusion_time.shape != (64,)):
                return None
            ps += [b.diffusion.diffusion_time, lins[0].weight, lins[0].bias, lins[1].weight, lins[1].bias,
                   lins[2].weight, lins[2].bias]
        ps += [self.last_lin.weight, self.last_lin.bias]
        if any(p is None for p in ps):
            return None
        return ps

    def forward(self, x_in, mass, L=None, evals=None, evecs=None, gradX=None, gradY=None, edges=None, faces=None):
        appended = x_in.dim() == 2
        if appended:
            x_in, mass, evals, evecs = x_in[None], mass[None], evals[None], evecs[None]
        ps = self._fused_params(x_in) if evecs is not None and evecs.shape[-1] == 64 else None
        if ps is not None and FUSED_ENCODER:
            x = _EncoderFn.apply(x_in.contiguous(), mass.contiguous(), evals.contiguous(), evecs.contiguous(),
                                 len(self.blocks), *ps)
            return x[0] if appended else x
        x = self.first_lin(x_in)
        for b in self.blocks:
            x = b(x, mass, L, evals, evecs, gradX, gradY)
        x = self.last_lin(x)
        if self.last_activation is not None:
            x = self.last_activation(x)
        return x[0] if appended else x
