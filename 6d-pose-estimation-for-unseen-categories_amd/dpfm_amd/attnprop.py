"""One fused autograd node per AttentionalPropagation call of the cross-attention refinement,
with its residual update (reference modeling/dpfm.py:45-82 and :101-103):

    desc' = desc + mlp(cat(desc, merge(attention(Pq desc, Pk src, Pv src))))

The module path (modeling/dpfm.py here) issues, per call, three projection launches, the
attention, the merge, a concatenation, the MLP (two layers + InstanceNorm/ReLU) and the residual
add forward; backward adds the slices' copies and the gradient accumulations of desc and src.
This node issues (forward) q, the stacked key/value projection (one 32 -> 64 launch reading
`src` once, pk_linear_ex w2), the attention on the stacked buffer (batch strides), the merge
written straight into the concatenation buffer, a copy of desc beside it (pk_copy_rows), mlp.0,
InstanceNorm+ReLU and mlp.3 with the residual in its epilogue; backward: mlp.3^T, the norm
backward, mlp.0^T, the merge^T reading its slice in place, the attention backward writing dk / dv
into one stacked buffer, Pq^T with BOTH other contributions to d desc (the residual and the
concatenation slice) added in its epilogue (add / add2), and [Pk; Pv]^T as one 64 -> 32 launch.
Weight gradients go to the grouped launch (layers.GroupedWgrad) reading the stacked / sliced
operands in place (pk_wgrad_call batch strides). Parameters and their names are the module's."""
from __future__ import annotations

import torch

from . import _lib, ops
from ._lib import call, ptr


def _wgrad(x, dy, weight, bias):
    """(dW, db) through the active GroupedWgrad, or computed here (None, None when recorded)."""
    from . import layers
    if layers._side_owns(weight, bias):
        layers._SIDE.launch(x, dy, weight, bias, channels_first=True)
        return None, None
    dw, db = ops.linear_wgrad(x, dy, channels_first=True, want_bias=bias is not None)
    return dw.view(weight.shape), db


def _prop_fwd(x, src, P, heads, eps):
    """desc' = x + layer(x, src) in the launches above; returns (desc', saved tensors)."""
    wq, bq, wk, bk, wv, bv, wm, bm, w0, b0, w3, b3 = P
    B, C, N = x.shape
    M = src.shape[2]
    D = C // heads
    dev = x.device
    f = lambda w: w.view(w.shape[0], -1)  # noqa: E731  Conv1d [O, I, 1] -> [O, I]
    q = torch.empty((B, C, N), dtype=torch.float32, device=dev)
    kv = torch.empty((B, 2 * C, M), dtype=torch.float32, device=dev)
    # the query and the stacked key / value projections: independent, one launch (pk_linear_ex2)
    ops.linear_ex2((x, f(wq), bq, 1, B * N, N, C, C, q), {},
                   (src, f(wk), bk, 1, B * M, M, C, 2 * C, kv), dict(w2=f(wv), bias2=bv, wsplit=C))
    a = torch.empty((B, C, N), dtype=torch.float32, device=dev)
    lse = torch.empty((B, heads, N, 2), dtype=torch.float32, device=dev)
    import ctypes
    vptr = ctypes.c_void_p(kv.data_ptr() + 4 * C * M)
    call("pk_attention_fwd", ptr(q), ptr(kv), vptr, B, D, heads, N, M, 2 * C * M, 2 * C * M, ptr(a), ptr(lse),
         _lib.stream(dev), work=("mfma", 2 * 2 * N * M * D * B * heads))
    hc = torch.empty((B, 2 * C, N), dtype=torch.float32, device=dev)  # cat(desc, message)
    call("pk_copy_rows", ptr(hc), 2 * C * N, ptr(x), C * N, B, C * N, _lib.stream(dev),
         work=("hbm", 8 * B * C * N))
    ops.linear_ex(a, f(wm), bm, 1, B * N, N, C, C, y=hc[:, C:], ldy=2 * C * N)
    h1 = torch.empty((B, 2 * C, N), dtype=torch.float32, device=dev)
    ops.linear_ex(hc, f(w0), b0, 1, B * N, N, 2 * C, 2 * C, y=h1)
    h1n = torch.empty_like(h1)
    mean = torch.empty((B * 2 * C,), dtype=torch.float32, device=dev)
    invstd = torch.empty_like(mean)
    call("pk_instnorm_relu_fwd", ptr(h1), B * 2 * C, N, float(eps), ptr(h1n), ptr(mean), ptr(invstd),
         _lib.stream(dev), work=("hbm", 8 * B * 2 * C * N))
    out = torch.empty((B, C, N), dtype=torch.float32, device=dev)
    ops.linear_ex(h1n, f(w3), b3, 1, B * N, N, 2 * C, C, y=out, add=x, add_cols=C)
    return out, (x, src, q, kv, a, lse, hc, h1, h1n, mean, invstd)


def _prop_bwd(saved, P, heads, dout, dsrc_add=None):
    """Gradients of one call: (d x, d src (+ dsrc_add, added in the launch's epilogue), the 12
    parameter gradients — None where the active GroupedWgrad takes them)."""
    x, src, q, kv, a, lse, hc, h1, h1n, mean, invstd = saved
    wq, bq, wk, bk, wv, bv, wm, bm, w0, b0, w3, b3 = P
    B, C, N = x.shape
    M = src.shape[2]
    D = C // heads
    dev = x.device
    f = lambda w: w.view(w.shape[0], -1)  # noqa: E731
    dout = dout.contiguous()
    # mlp.3 (its residual: dout flows to desc unchanged, added in Pq^T's epilogue below)
    dh1n = torch.empty((B, 2 * C, N), dtype=torch.float32, device=dev)
    ops.linear_ex(dout, f(w3), None, 1, B * N, N, C, 2 * C, y=dh1n, transw=True)
    g_w3, g_b3 = _wgrad(h1n, dout, w3, b3)
    dh1 = torch.empty_like(dh1n)
    call("pk_instnorm_relu_bwd", ptr(h1), ptr(dh1n), ptr(mean), ptr(invstd), B * 2 * C, N, ptr(dh1),
         _lib.stream(dev), work=("hbm", 12 * B * 2 * C * N))
    dhc = torch.empty((B, 2 * C, N), dtype=torch.float32, device=dev)
    ops.linear_ex(dh1, f(w0), None, 1, B * N, N, 2 * C, 2 * C, y=dhc, transw=True)
    g_w0, g_b0 = _wgrad(hc, dh1, w0, b0)
    # merge^T on the message half of the concatenation gradient, read in place
    da = torch.empty((B, C, N), dtype=torch.float32, device=dev)
    ops.linear_ex(dhc[:, C:], f(wm), None, 1, B * N, N, C, C, y=da, transw=True, ldx=2 * C * N)
    g_wm, g_bm = _wgrad(a, dhc[:, C:], wm, bm)
    # attention backward: dk / dv into one stacked buffer
    dq = torch.empty((B, C, N), dtype=torch.float32, device=dev)
    dkv = torch.empty((B, 2 * C, M), dtype=torch.float32, device=dev)
    work = ops.attention_bwd_work(B, D, heads, N, M, dev)
    import ctypes
    off = 4 * C * M
    call("pk_attention_bwd", ptr(q), ptr(kv), ctypes.c_void_p(kv.data_ptr() + off), ptr(a), ptr(da), ptr(lse),
         B, D, heads, N, M, 2 * C * M, 2 * C * M, ptr(work), ptr(dq), ptr(dkv),
         ctypes.c_void_p(dkv.data_ptr() + off), 2 * C * M, 2 * C * M, _lib.stream(dev),
         work=("mfma", 5 * 2 * N * M * D * B * heads))  # S, dP, dV, dK, dQ: each contraction once
    # d desc = Pq^T dq + dout (residual) + dhc[:, :C] (concatenation) and d src = Pk^T dk + Pv^T dv
    # (+ the source's other gradient; the stacked weight's transpose, 64 -> 32): independent, one
    # launch (pk_linear_ex2)
    dx = torch.empty((B, C, N), dtype=torch.float32, device=dev)
    dsrc = torch.empty((B, C, M), dtype=torch.float32, device=dev)
    if dsrc_add is not None:
        dsrc_add = dsrc_add.contiguous()
    ops.linear_ex2((dq, f(wq), None, 1, B * N, N, C, C, dx),
                   dict(transw=True, add=dout, add_cols=C, add2=dhc[:, :C], lda2=2 * C * N),
                   (dkv, f(wk), None, 1, B * M, M, 2 * C, C, dsrc),
                   dict(transw=True, w2=f(wv), wsplit=C, add=dsrc_add, add_cols=C if dsrc_add is not None else 0))
    g_wq, g_bq = _wgrad(x, dq, wq, bq)
    g_wk, g_bk = _wgrad(src, dkv[:, :C], wk, bk)
    g_wv, g_bv = _wgrad(src, dkv[:, C:], wv, bv)
    return dx, dsrc, [g_wq, g_bq, g_wk, g_bk, g_wv, g_bv, g_wm, g_bm, g_w0, g_b0, g_w3, g_b3]


class _AttnPropFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, src, wq, bq, wk, bk, wv, bv, wm, bm, w0, b0, w3, b3, heads, eps):
        P = (wq, bq, wk, bk, wv, bv, wm, bm, w0, b0, w3, b3)
        out, saved = _prop_fwd(x, src, P, heads, eps)
        ctx.heads = heads
        ctx.params = P
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, dout):
        dx, dsrc, g = _prop_bwd(ctx.saved_tensors, ctx.params, ctx.heads, dout)
        return (dx, dsrc, *g, None, None)


class _AttnPropPairFn(torch.autograd.Function):
    """One refinement layer's two calls (modeling/dpfm.py:101-103) as one node:
        out0 = x0 + layer(x0, x1);  out1 = x1 + layer(x1, out0)
    so each gradient that two consumers feed is summed in a launch epilogue instead of by the
    autograd engine: d out0 = g0 + (the second call's d src) in that launch's `add`, d x1 =
    (the second call's d x) + (the first call's d src) likewise. Parameter gradients: the second
    call's, then the first's, autograd's order for a layer applied twice."""

    @staticmethod
    def forward(ctx, x0, x1, wq, bq, wk, bk, wv, bv, wm, bm, w0, b0, w3, b3, heads, eps):
        P = (wq, bq, wk, bk, wv, bv, wm, bm, w0, b0, w3, b3)
        out0, s0 = _prop_fwd(x0, x1, P, heads, eps)
        out1, s1 = _prop_fwd(x1, out0, P, heads, eps)
        ctx.heads = heads
        ctx.params = P
        ctx.save_for_backward(*s0, *s1)
        return out0, out1

    @staticmethod
    def backward(ctx, g0, g1):
        sv = ctx.saved_tensors
        s0, s1 = sv[:11], sv[11:]
        dx1_b, dout0, gb = _prop_bwd(s1, ctx.params, ctx.heads, g1, dsrc_add=g0)
        dx0, dx1, ga = _prop_bwd(s0, ctx.params, ctx.heads, dout0, dsrc_add=dx1_b)
        g = [b if a is None else (a if b is None else b + a) for a, b in zip(ga, gb)]
        return (dx0, dx1, *g, None, None)


def _fusable(layer, x, src) -> bool:
    attn, mlp = layer.attn, layer.mlp
    C = x.shape[1] if x.dim() == 3 else 0
    return (x.is_cuda and x.dim() == 3 and src.dim() == 3 and x.is_contiguous() and src.is_contiguous()
            and x.dtype == torch.float32 and src.dtype == torch.float32 and C in (16, 32, 64)
            and attn.dim == 16 and C == attn.dim * attn.num_heads and len(mlp) == 4
            and x.shape[0] == src.shape[0] and src.shape[1] == C
            and mlp[0].out_channels == 2 * C and mlp[3].out_channels == C)


def _params(layer):
    attn, mlp = layer.attn, layer.mlp
    pq, pk, pv = attn.proj
    return (pq.weight, pq.bias, pk.weight, pk.bias, pv.weight, pv.bias, attn.merge.weight, attn.merge.bias,
            mlp[0].weight, mlp[0].bias, mlp[3].weight, mlp[3].bias)


def attn_prop_pair(layer, x0: torch.Tensor, x1: torch.Tensor):
    """(x0', x1') = (x0 + layer(x0, x1), x1 + layer(x1, x0')) — both calls of one refinement layer
    (modeling/dpfm.py:101-103) as one fused node — or None outside the fused shapes."""
    if not (_fusable(layer, x0, x1) and _fusable(layer, x1, x0)):
        return None
    return _AttnPropPairFn.apply(x0, x1, *_params(layer), layer.attn.num_heads, float(layer.mlp[1].eps))


def attn_prop_residual(layer, x: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """x + layer(x, src) for a modeling.dpfm.AttentionalPropagation `layer` as one fused node, or
    None when the shapes / storage fall outside it (the caller then takes the module path)."""
    if not _fusable(layer, x, src):
        return None
    return _AttnPropFn.apply(x, src, *_params(layer), layer.attn.num_heads, float(layer.mlp[1].eps))
