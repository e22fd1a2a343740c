"""DPFMNet — drop-in for reference models/dpfm.py:15-82.

`DPFMNet(cfg).forward(batch)` keeps the reference contract: cfg is the parsed
config/dpfm_orig.yaml dict, batch = {"shape1": CAD, "shape2": PC} with xyz / mass /
evals / evecs (L, gradX, gradY, faces accepted and unused, as in the reference's
spectral configuration); returns (C_pred, overlap12, overlap21, use_feat1, use_feat2,
ref_feat1, ref_feat2). state_dict keys equal weights/weights.pt.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from ..diffusion_net import DiffusionNet
from ..modeling.dpfm import CrossAttentionRefinementNet, RegularizedFMNet

# models/dpfm.py:66-72 + RegularizedFMNet as the fused two-launch head (ops.fmap_head); False runs
# the per-module path (the parity tests compare the two)
FUSED_FMAP_HEAD = True

DEFAULT_CFG = {  # config/dpfm_orig.yaml
    "fmap": {"n_fmap": 30, "k_eig": 64, "n_feat": 32, "C_in": 3, "lambda_": 100, "resolvant_gamma": 0.5,
             "robust": True},
    "attention": {"num_head": 2, "gnn_dim": 32, "ref_n_layers": 1, "cross_sampling_ratio": 1.0,
                  "attention_type": "normal"},
    "overlap": {"overlap_feat_dim": 32},
}


def _cat0(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """torch.cat((a, b), 0), without a copy when b directly follows a in one storage (the
    device pipeline keeps the CAD and crop operators of a batch in one buffer)."""
    if (a.is_contiguous() and b.is_contiguous() and a.dtype == b.dtype and a.device == b.device
            and a.shape[1:] == b.shape[1:]
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
            and b.storage_offset() == a.storage_offset() + a.numel()):
        return a.as_strided((a.shape[0] + b.shape[0],) + tuple(a.shape[1:]), a.stride())
    return torch.cat((a, b), 0)


class DPFMNet(nn.Module):
    """Compute the functional map matrix representation."""

    def __init__(self, cfg=None):
        super().__init__()
        cfg = cfg or DEFAULT_CFG
        self.feature_extractor = DiffusionNet(C_in=cfg["fmap"]["C_in"], C_out=cfg["fmap"]["n_feat"], C_width=64,
                                              N_block=2, dropout=False, with_gradient_features=False,
                                              with_gradient_rotations=True)
        a = cfg["attention"]
        self.feat_refiner = CrossAttentionRefinementNet(
            n_in=cfg["fmap"]["n_feat"], num_head=a["num_head"], gnn_dim=a["gnn_dim"],
            overlap_feat_dim=cfg["overlap"]["overlap_feat_dim"], n_layers=a["ref_n_layers"],
            cross_sampling_ratio=a["cross_sampling_ratio"], attention_type=a["attention_type"])
        self.fmreg_net = RegularizedFMNet(lambda_=cfg["fmap"]["lambda_"], resolvant_gamma=cfg["fmap"]["resolvant_gamma"])
        self.n_fmap = cfg["fmap"]["n_fmap"]
        self.robust = cfg["fmap"]["robust"]

    def forward(self, batch):
        s1, s2 = batch["shape1"], batch["shape2"]
        verts1, mass1, evals1, evecs1 = s1["xyz"], s1["mass"], s1["evals"], s1["evecs"]
        verts2, mass2, evals2, evecs2 = s2["xyz"], s2["mass"], s2["evals"], s2["evecs"]
        if verts1.dim() == 3 and verts1.shape == verts2.shape and evecs1.shape == evecs2.shape:
            # same weights, per-crop operations: one pass over both shapes (2B crops); the
            # input features (v - 110) / 50 of both shapes (models/dpfm.py:53) in one launch
            B = verts1.shape[0]
            if verts1.is_cuda and verts1.dtype == torch.float32 and not verts1.requires_grad:
                fcat = ops.affine_cat(verts1, verts2, 110.0, 50.0)
            else:
                fcat = torch.cat(((verts1 - 110) / 50, (verts2 - 110) / 50), 0)
            feat = self.feature_extractor(fcat, _cat0(mass1, mass2),
                                          evals=_cat0(evals1, evals2), evecs=_cat0(evecs1, evecs2))
            feat1, feat2 = torch.chunk(feat, 2, 0)  # (the refiner's first_lin reads feat whole)
            fused_cat = True
        else:
            fused_cat = False
            features1, features2 = (verts1 - 110) / 50, (verts2 - 110) / 50  # models/dpfm.py:53
            feat1 = self.feature_extractor(features1, mass1, evals=evals1, evecs=evecs1)
            feat2 = self.feature_extractor(features2, mass2, evals=evals2, evecs=evecs2)

        ref_feat1, ref_feat2, overlap_score12, overlap_score21 = self.feat_refiner(
            verts1, verts2, feat1, feat2, batch, features_xy=feat if fused_cat else None)
        use_feat1, use_feat2 = (ref_feat1, ref_feat2) if self.robust else (feat1, feat2)

        k = self.n_fmap
        if (evecs1.dim() == 3 and evecs1.is_cuda and k == 30 and use_feat1.shape[-1] == 32
                and FUSED_FMAP_HEAD):
            # models/dpfm.py:66-72 + RegularizedFMNet (modeling/dpfm.py:154-195) fused: the
            # projections, AAt / BAt, the resolvent mask and the solve in two launches
            C_pred = ops.fmap_head(use_feat1, use_feat2, evecs1, evecs2, mass1, mass2, evals1, evals2,
                                   self.fmreg_net.lambda_, self.fmreg_net.resolvant_gamma)
            return C_pred, overlap_score12, overlap_score21, use_feat1, use_feat2, ref_feat1, ref_feat2
        if evecs1.dim() == 3:  # models/dpfm.py:66-72, batched instead of a loop over crops
            evecs_trans1 = (evecs1[:, :, :k] * mass1[:, :, None]).transpose(1, 2)
            evecs_trans2 = (evecs2[:, :, :k] * mass2[:, :, None]).transpose(1, 2)
            ev1, ev2 = evals1[:, :k], evals2[:, :k]
        else:
            evecs_trans1 = (evecs1[:, :k] * mass1[:, None]).t()
            evecs_trans2 = (evecs2[:, :k] * mass2[:, None]).t()
            ev1, ev2 = evals1[:k], evals2[:k]
        C_pred = self.fmreg_net(use_feat1, use_feat2, ev1, ev2, evecs_trans1, evecs_trans2)
        return C_pred, overlap_score12, overlap_score21, use_feat1, use_feat2, ref_feat1, ref_feat2
