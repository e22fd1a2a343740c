"""DPFM training loss (reference utils/loss.py:8-99 + upstream WeightedBCELoss), batched
over crops on the device: no per-crop Python loop, no host syncs (the reference's
`.item()` logging is produced lazily by `as_log`)."""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..dpfm_utils import FrobeniusLoss

__all__ = ["FrobeniusLoss", "NCESoftmaxLoss", "DPFMLoss", "nce_select"]


_NCE_CTR: dict = {}


def nce_select(counts: torch.Tensor, cap: int, num: int, generator: Optional[torch.Generator] = None):
    """Per crop, `num` distinct pair rows drawn uniformly without replacement when the crop
    has more than `num` pairs, all rows otherwise (utils/loss.py:27-30). Returns
    (rows int64 [B, min(num, cap)], valid bool [B, min(num, cap)]).

    Drawn by pk_nce_select (keyed bijection on the device: no sort, no memset, no host
    RNG, so it can sit inside a HIP graph). The key is the generator's seed plus a
    device step counter owned by that generator, advanced by every call."""
    from .. import ops
    dev = counts.device
    seed = int(generator.initial_seed()) if generator is not None else 0
    key = (id(generator), str(dev))
    ctr = _NCE_CTR.get(key)
    if ctr is None:
        ctr = _NCE_CTR[key] = torch.zeros(1, dtype=torch.int64, device=dev)
    return ops.nce_select(counts.to(torch.int64).contiguous(), int(cap), int(num), seed, ctr)


class NCESoftmaxLoss(nn.Module):
    def __init__(self, nce_t, nce_num_pairs):
        super().__init__()
        self.nce_t = nce_t
        self.nce_num_pairs = nce_num_pairs

    def forward_batched(self, f1, f2, pairs, rows, valid):
        """Per-crop NCE loss [B]: pairs [B, cap, 2], rows/valid from nce_select; one fused
        kernel pair (ops.nce_loss)."""
        from .. import ops
        if not f1.is_cuda:
            raise ops._lib.PoseKernError("NCESoftmaxLoss runs on HIP devices only (no CPU fallback)")
        return ops.nce_loss(f1, f2, pairs, rows, valid, self.nce_t)

    def forward_batched_torch(self, f1, f2, pairs, rows, valid):
        """The same per-crop NCE loss composed of torch ops (development comparison only;
        the training step uses the fused kernel above)."""
        f1n, f2n = F.normalize(f1, p=2, dim=-1), F.normalize(f2, p=2, dim=-1)
        sel = torch.gather(pairs, 1, rows[..., None].expand(-1, -1, 2))
        # rows past a crop's pair count select unwritten slots of the pair buffer: point
        # them at row 0 so the feature gathers stay in bounds (their terms are masked)
        sel = torch.where(valid[..., None], sel, torch.zeros_like(sel))
        q = torch.gather(f1n, 1, sel[..., 0:1].expand(-1, -1, f1n.shape[-1]))
        k = torch.gather(f2n, 1, sel[..., 1:2].expand(-1, -1, f2n.shape[-1]))
        logits = -torch.cdist(q, k) / self.nce_t
        logits = logits.masked_fill(~valid[:, None, :], float("-inf"))
        logp = torch.log_softmax(logits, dim=-1)
        diag = torch.diagonal(logp, dim1=1, dim2=2)
        diag = torch.where(valid, diag, torch.zeros_like(diag))
        return -diag.sum(1) / valid.sum(1).clamp(min=1)

    def forward(self, features_1, features_2, map21, generator=None):
        """Reference signature (utils/loss.py:22): one crop, map21 int [P, 2]."""
        dev = features_1.device
        pairs = map21.to(device=dev, dtype=torch.int64)[None]
        cnt = torch.tensor([pairs.shape[1]], device=dev)
        rows, valid = nce_select(cnt, pairs.shape[1], self.nce_num_pairs, generator)
        return self.forward_batched(features_1.squeeze(0)[None], features_2.squeeze(0)[None], pairs, rows, valid)[0]


class _BCE(torch.autograd.Function):
    """F.binary_cross_entropy(reduction='none') with ATen's formulas (log terms clamped at
    -100; gradient (x - t) / max(x (1 - x), 1e-12)) but without the library kernel's
    device-side range assert, which inside a HIP graph aborts the whole queue instead of
    surfacing as a NaN loss."""

    @staticmethod
    def forward(ctx, x, t):
        ctx.save_for_backward(x, t)
        return (t - 1) * torch.clamp(torch.log1p(-x), min=-100) - t * torch.clamp(torch.log(x), min=-100)

    @staticmethod
    def backward(ctx, g):
        x, t = ctx.saved_tensors
        return g * (x - t) / torch.clamp((1 - x) * x, min=1e-12), None


def weighted_bce_batched(pred, gt):
    """Upstream WeightedBCELoss per crop: pred/gt [B, N] -> [B] (padding counts, as in the
    reference where collate pads the overlap masks)."""
    loss = _BCE.apply(pred, gt)
    w_neg = gt.sum(1, keepdim=True) / gt.shape[1]
    w = torch.where(gt >= 0.5, 1 - w_neg, w_neg)
    return (w * loss).mean(1)


class DPFMLoss(nn.Module):
    def __init__(self, w_fmap=1, w_acc=1, w_nce=0.1, nce_t=0.07, nce_num_pairs=4096):
        super().__init__()
        self.w_fmap, self.w_acc, self.w_nce = w_fmap, w_acc, w_nce
        self.frob_loss = FrobeniusLoss()
        self.nce_softmax_loss = NCESoftmaxLoss(nce_t, nce_num_pairs)

    def forward_batched(self, C12, C_gt, pairs, npairs, feat1, feat2, o12, o21, gt12, gt21,
                        generator: Optional[torch.Generator] = None, selection=None):
        """All crops at once. pairs int64 [B, cap, 2] (CAD idx, PC idx), npairs [B];
        returns (loss, dict of 0-d tensors). One autograd node (ops.dpfm_loss): the NCE and
        WBCE kernels with their input gradients plus the fused scalar head."""
        from .. import ops
        if not C12.is_cuda:
            raise ops._lib.PoseKernError("DPFMLoss runs on HIP devices only (no CPU fallback)")
        if o12.dim() == 1:
            o12, o21 = o12[None], o21[None]
        rows, valid = selection if selection is not None else nce_select(
            npairs, pairs.shape[1], self.nce_softmax_loss.nce_num_pairs, generator)
        loss, logs = ops.dpfm_loss(C12, C_gt, feat1, feat2, pairs, rows, valid, o12, o21, gt12, gt21,
                                   self.w_fmap, self.w_acc, self.w_nce, self.nce_softmax_loss.nce_t)
        return loss, {"nce_loss": logs[0], "acc_loss": logs[1], "fmap_loss": logs[2], "loss": loss.detach()}

    def forward_batched_composed(self, C12, C_gt, pairs, npairs, feat1, feat2, o12, o21, gt12, gt21,
                                 generator: Optional[torch.Generator] = None, selection=None):
        """The same loss composed from the per-term kernels and torch ops (development
        comparison for the fused head)."""
        fmap_loss = self.frob_loss(C12, C_gt) * self.w_fmap
        m = feat1.shape[0]
        if o12.dim() == 1:
            o12, o21 = o12[None], o21[None]
        rows, valid = selection if selection is not None else nce_select(
            npairs, pairs.shape[1], self.nce_softmax_loss.nce_num_pairs, generator)
        nce = self.nce_softmax_loss.forward_batched(feat1, feat2, pairs, rows, valid)
        nce_loss = (nce * self.w_nce / m).sum()
        from .. import ops
        wb = ops.weighted_bce_pair(o12, o21, gt12, gt21)  # both directions, loss + gradient, one launch
        acc_loss = ((wb[0] + wb[1]) * self.w_acc / m).sum()
        loss = fmap_loss + acc_loss + nce_loss
        return loss, {"nce_loss": nce_loss.detach(), "acc_loss": acc_loss.detach(),
                      "fmap_loss": fmap_loss.detach(), "loss": loss.detach()}

    def forward(self, C12, C_gt, map21: Sequence[torch.Tensor], feat1, feat2, overlap_score12, overlap_score21,
                gt_partiality_mask12, gt_partiality_mask21):
        """Reference signature (utils/loss.py:57): map21 is a list of [P_b, 2] pair lists."""
        dev = feat1.device
        cnt = torch.tensor([int(p.shape[0]) for p in map21], device=dev)
        cap = max(1, int(cnt.max().item()))
        pairs = torch.zeros((len(map21), cap, 2), dtype=torch.int64, device=dev)
        for b, p in enumerate(map21):
            pairs[b, :p.shape[0]] = torch.as_tensor(p, device=dev).to(torch.int64)
        loss, log = self.forward_batched(C12, C_gt, pairs, cnt, feat1, feat2, overlap_score12, overlap_score21,
                                         gt_partiality_mask12, gt_partiality_mask21)
        return loss, {k: float(v) for k, v in log.items()}
