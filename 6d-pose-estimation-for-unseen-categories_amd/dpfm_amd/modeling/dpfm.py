"""Cross-attention refinement, overlap head and regularized fmap head (H8, H9).

Mirror of reference modeling/dpfm.py:16-195: same classes, constructor arguments,
parameter names (weights/weights.pt loads strictly) and semantics, including the
reference's quirks: heads interleaved by view(B, dim, heads, N)
(:53), desc1 updated with the already-updated desc0 (:101-103), unmasked
InstanceNorm over zero padding (:24), the batched fmap branch always taken (:164).
The attention core runs in the fused HIP kernel `ops.attention` (scores never hit HBM);
the 30 sequential inverses of the fmap head are one HIP launch (`ops.fmap_solve`).
"""
from __future__ import annotations

from copy import deepcopy

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..layers import Conv1d, Linear, pointwise_residual
from ..dpfm_utils import get_mask_batched


class InstanceNormReLU(nn.InstanceNorm1d):
    """nn.InstanceNorm1d(C) (affine=False, no running stats: no parameters or buffers, so
    state_dict keys are unchanged) followed by the ReLU of the next Sequential slot, fused in
    one HIP kernel per direction (ops.instnorm_relu); the slot after it holds an Identity so
    the Sequential's indices (mlp.0 / mlp.3) match the reference's."""

    def forward(self, x):
        if self.affine or self.track_running_stats:
            raise ValueError("the reference's InstanceNorm1d is affine=False, track_running_stats=False")
        return ops.instnorm_relu(x, self.eps)


FUSED_ATTN_PROP = True  # AttentionalPropagation + residual as one fused node (attnprop.py)
FUSED_OVERLAP_HEAD = True  # OverlapPredictorNet for both shapes as one fused node (ops.overlap_head)


def MLP(channels: list, do_bn=True):
    """Multi-layer perceptron of 1x1 convolutions (modeling/dpfm.py:16-26)."""
    n = len(channels)
    layers = []
    for i in range(1, n):
        layers.append(Conv1d(channels[i - 1], channels[i], kernel_size=1, bias=True))
        if i < (n - 1):
            if do_bn:
                layers.append(InstanceNormReLU(channels[i]))
                layers.append(nn.Identity())  # the ReLU, applied inside InstanceNormReLU
            else:
                layers.append(nn.ReLU())
    return nn.Sequential(*layers)


def attention(query, key, value):
    """modeling/dpfm.py:29-37. Tensors are [B, d, heads, N]; returns (result, None): the
    probability matrix is never materialised (the reference's caller discards it)."""
    return ops.attention(query, key, value), None


class MultiHeadedAttention(nn.Module):
    def __init__(self, num_heads: int, d_model: int):
        super().__init__()
        assert d_model % num_heads == 0
        self.dim = d_model // num_heads
        self.num_heads = num_heads
        self.merge = Conv1d(d_model, d_model, kernel_size=1)
        self.proj = nn.ModuleList([deepcopy(self.merge) for _ in range(3)])

    def forward(self, query, key, value):
        B = query.size(0)
        q, k, v = [ll(x).view(B, self.dim, self.num_heads, -1) for ll, x in zip(self.proj, (query, key, value))]
        x, _ = attention(q, k, v)
        return self.merge(x.contiguous().view(B, self.dim * self.num_heads, -1))


class AttentionalPropagation(nn.Module):
    def __init__(self, feature_dim: int, num_heads: int):
        super().__init__()
        self.attn = MultiHeadedAttention(num_heads, feature_dim)
        self.mlp = MLP([feature_dim * 2, feature_dim * 2, feature_dim])
        nn.init.constant_(self.mlp[-1].bias, 0.0)

    def forward(self, x, source):
        message = self.attn(x, source, source)
        return self.mlp(torch.cat([x, message], dim=1))

    def forward_residual(self, x, source):
        """x + forward(x, source) (modeling/dpfm.py:101-103's residual update): one fused autograd
        node (attnprop.attn_prop_residual) where the shapes allow, else the module path with the
        add folded into the MLP's last layer (layers.pointwise_residual)."""
        if FUSED_ATTN_PROP:
            from ..attnprop import attn_prop_residual
            y = attn_prop_residual(self, x, source)
            if y is not None:
                return y
        message = self.attn(x, source, source)
        h = self.mlp[:-1](torch.cat([x, message], dim=1))
        return pointwise_residual(self.mlp[-1], h, x)


class CrossAttentionRefinementNet(nn.Module):
    def __init__(self, n_in=128, num_head=4, gnn_dim=512, overlap_feat_dim=32, n_layers=2,
                 cross_sampling_ratio=0.15, attention_type="normal"):
        super().__init__()
        self.attention_type = attention_type
        if attention_type == "normal":
            additional_dim = 0
            overlap_feat_dim = n_in
        elif attention_type == "double":
            additional_dim = overlap_feat_dim
        else:
            raise Exception("Attention type not recognized")
        if cross_sampling_ratio != 1:
            # the subsampled branch (modeling/dpfm.py:105-118) references undefined names in
            # the reference and can never run; only ratio 1.0 is a working configuration
            raise ValueError("cross_sampling_ratio != 1 is not a working configuration of the reference")
        self.n_in = n_in
        self.cross_sampling_ratio = cross_sampling_ratio
        self.layers = nn.ModuleList([AttentionalPropagation(gnn_dim + additional_dim, num_head) for _ in range(n_layers)])
        self.first_lin = Linear(n_in, gnn_dim + additional_dim)
        self.first_lin.out_cf = True  # desc = first_lin(x).transpose(1, 2) is then contiguous
        self.last_lin = Linear(gnn_dim + additional_dim, n_in + additional_dim)
        self.overlap_predictor = OverlapPredictorNet(overlap_feat_dim=overlap_feat_dim)

    def forward(self, coords0, coords1, features_x, features_y, batch=None, features_xy=None):
        """features_xy (optional): the encoder's [2B, N, C] output of which features_x / features_y
        are the two halves; first_lin then runs once on it (layers.linear_pair_cf)."""
        pair = None
        if features_xy is not None and FUSED_ATTN_PROP:
            from ..layers import linear_pair_cf
            pair = linear_pair_cf(self.first_lin, features_xy, features_x.shape[0])
        if pair is not None:
            desc0, desc1 = pair
        else:
            desc0, desc1 = self.first_lin(features_x).transpose(1, 2), self.first_lin(features_y).transpose(1, 2)
        for layer in self.layers:
            pair = None
            if FUSED_ATTN_PROP:  # both calls of the layer as one node (attnprop.attn_prop_pair)
                from ..attnprop import attn_prop_pair
                pair = attn_prop_pair(layer, desc0, desc1)
            if pair is not None:
                desc0, desc1 = pair
            else:
                desc0 = layer.forward_residual(desc0, desc1)
                desc1 = layer.forward_residual(desc1, desc0)  # with the updated desc0 (:101-103)
        op = self.overlap_predictor
        ll = self.last_lin
        if (FUSED_ATTN_PROP and self.attention_type == "normal" and ll.out_features == self.n_in
                and not ll.relu_out and not ll.sigmoid_out and desc0.is_contiguous() and desc1.is_contiguous()
                and desc0.dim() == 3 and ll.in_features == desc0.shape[1] == desc1.shape[1]
                and ll.in_features in (16, 32, 64, 128)
                and op._fusable(desc0.transpose(1, 2)[..., :self.n_in], desc1.transpose(1, 2)[..., :self.n_in])):
            # last_lin + the overlap head as one node: the refined features' two consumers (the
            # overlap head here, the fmap head downstream) meet in one launch's epilogue
            l0, l2 = op.overlap_score_net[0], op.overlap_score_net[2]
            y0, y1, sx, sy, rx, ry = ops.lastlin_overlap_head(desc0, desc1, ll.weight, ll.bias, l0.weight, l0.bias,
                                                              l2.weight, l2.bias)
            ref_x, ref_y = y0.transpose(1, 2), y1.transpose(1, 2)
            if rx is not None:
                ref_x._pk_nrows, ref_y._pk_nrows = rx, ry
            return ref_x, ref_y, sx.squeeze(0), sy.squeeze(0)
        ax = self.last_lin(desc0.transpose(1, 2))
        ay = self.last_lin(desc1.transpose(1, 2))
        if ax.shape[-1] == self.n_in:  # "normal" attention: the whole width (no slice, whose
            ref_x, ref_y = ax, ay     # backward would zero-fill and copy)
        else:
            ref_x, ref_y = ax[:, :, :self.n_in], ay[:, :, :self.n_in]
        if self.attention_type == "normal":
            ox, oy = self.overlap_predictor(ref_x, ref_y)
        else:
            ox, oy = self.overlap_predictor(ax[:, :, self.n_in:], ay[:, :, self.n_in:])
        return ref_x, ref_y, ox, oy


class OverlapPredictorNet(nn.Module):
    def __init__(self, overlap_feat_dim=32):
        super().__init__()
        self.overlap_score_net = nn.Sequential(
            Linear(overlap_feat_dim, overlap_feat_dim, bias=True),
            nn.Identity(),  # the reference's nn.ReLU(True), applied in layer 0's epilogue
            Linear(overlap_feat_dim, 1, bias=True),
            nn.Identity(),  # the reference's nn.Sigmoid(), applied in layer 2's epilogue
        )
        self.overlap_score_net[0].relu_out = True
        self.overlap_score_net[2].sigmoid_out = True

    def _fusable(self, fx, fy) -> bool:
        l0, l2 = self.overlap_score_net[0], self.overlap_score_net[2]
        return (FUSED_OVERLAP_HEAD and fx.is_cuda and fx.dim() == 3 and fy.dim() == 3 and fx.shape[-1] == 32
                and fy.shape[-1] == 32 and fx.shape[0] == fy.shape[0] and fx.dtype == torch.float32
                and fy.dtype == torch.float32 and tuple(l0.weight.shape) == (32, 32) and tuple(l2.weight.shape) == (1, 32)
                and l0.bias is not None and l2.bias is not None and l0.relu_out and l2.sigmoid_out)

    def forward(self, overlap_feat_x, overlap_feat_y):
        if self._fusable(overlap_feat_x, overlap_feat_y):
            # the whole head for both shapes in one launch per direction (ops.overlap_head); the
            # rows copies of the normalized features go to the loss's NCE term as below
            l0, l2 = self.overlap_score_net[0], self.overlap_score_net[2]
            sx, sy, rx, ry = ops.overlap_head(overlap_feat_x, overlap_feat_y, l0.weight, l0.bias, l2.weight, l2.bias)
            if rx is not None:
                overlap_feat_x._pk_nrows, overlap_feat_y._pk_nrows = rx, ry
            return sx.squeeze(0), sy.squeeze(0)  # [B, N] = the reference's [B, N, 1].squeeze(2).squeeze(0)
        # F.normalize(., p=2, dim=-1) (modeling/dpfm.py:140-141), fused, storage order kept; a rows
        # copy of the normalized features is attached to the input for the loss's NCE term
        # (the same normalization, utils/loss.py:23-24), which then reads whole rows
        nx = ny = None
        if (torch.is_grad_enabled() and overlap_feat_x.dim() == 3 and overlap_feat_x.is_cuda
                and overlap_feat_x.shape[-1] == 32):
            nx, overlap_feat_x._pk_nrows = ops.l2_normalize_two(overlap_feat_x)
            ny, overlap_feat_y._pk_nrows = ops.l2_normalize_two(overlap_feat_y)
        if nx is None:
            nx = ops.l2_normalize(overlap_feat_x) if overlap_feat_x.dim() == 3 else F.normalize(overlap_feat_x, p=2, dim=-1)
            ny = ops.l2_normalize(overlap_feat_y) if overlap_feat_y.dim() == 3 else F.normalize(overlap_feat_y, p=2, dim=-1)
        sx = self.overlap_score_net(nx).squeeze(2).squeeze(0)
        sy = self.overlap_score_net(ny).squeeze(2).squeeze(0)
        return sx, sy


class RegularizedFMNet(nn.Module):
    """Compute the functional map matrix representation (modeling/dpfm.py:154-195)."""

    def __init__(self, lambda_=1e-3, resolvant_gamma=0.5):
        super().__init__()
        self.lambda_ = lambda_
        self.resolvant_gamma = resolvant_gamma

    def forward(self, feat_x, feat_y, evals_x, evals_y, evecs_trans_x, evecs_trans_y):
        # the reference compares the bound method `.dim` with 2 (:164), so the batched
        # branch below is the one that always runs
        if evecs_trans_x.dim() == 2:
            evecs_trans_x, evecs_trans_y = evecs_trans_x[None], evecs_trans_y[None]
            evals_x, evals_y = evals_x[None], evals_y[None]
        A = torch.bmm(evecs_trans_x, feat_x)
        Bm = torch.bmm(evecs_trans_y, feat_y)
        with torch.no_grad():  # per-crop get_mask (:171-176), batched, one launch
            ex, ey = evals_x.flatten(1), evals_y.flatten(1)
            if ex.is_cuda and ex.dtype == torch.float32 and ex.shape == ey.shape and ex.shape[1] <= 32:
                D = ops.resolvent_mask(ex, ey, self.resolvant_gamma)
            else:
                D = get_mask_batched(ex, ey, self.resolvant_gamma)
        A_t = A.transpose(1, 2)
        return ops.fmap_solve(torch.bmm(A, A_t), torch.bmm(Bm, A_t), D, self.lambda_)
