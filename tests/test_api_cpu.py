"""CPU: API surface of the drop-in (names, shapes, reference signatures)."""
import inspect

import torch

from oracle import dpfm_model_oracle as M


def test_weights_pt_state_dict_names():
    """The product model exposes exactly the reference's parameter names/shapes."""
    from dpfm_amd.models.dpfm import DPFMNet
    ref = M.DPFMNet().state_dict()
    mine = DPFMNet().state_dict()
    assert {k: tuple(v.shape) for k, v in ref.items()} == {k: tuple(v.shape) for k, v in mine.items()}
    assert sum(v.numel() for v in mine.values()) == 49281


def test_reference_signatures():
    from dpfm_amd.dataset import object as obj
    from dpfm_amd.fmap2pointmap_solvers import naive_fmap2pointmap, spacial_filtering_fmap2pointmap
    from dpfm_amd.pose.ransac import ransac_registration
    from dpfm_amd.utils import C_from_sparse_P, compute_inlier_ratio
    from dpfm_amd.dpfm_utils import farthest_point_sample
    assert list(inspect.signature(obj.find_positives).parameters)[:3] == ["pc1", "pc2", "r"]
    assert list(inspect.signature(obj.dpt_2_pcld).parameters)[:4] == ["dpt", "cam_scale", "K", "mask"]
    assert list(inspect.signature(obj.transform).parameters)[:4] == ["pc", "R", "t", "inv"]
    assert list(inspect.signature(spacial_filtering_fmap2pointmap).parameters) == [
        "C12", "evecs_x", "evecs_y", "CAD", "PC", "diam_cad"]
    assert list(inspect.signature(naive_fmap2pointmap).parameters)[:3] == ["C12", "evecs_x", "evecs_y"]
    assert list(inspect.signature(ransac_registration).parameters)[:5] == [
        "cad_xyz", "pc_xyz", "P", "distance_threshold", "num_iterations"]
    assert list(inspect.signature(C_from_sparse_P).parameters) == ["P", "evecs1", "evecs2"]
    assert list(inspect.signature(compute_inlier_ratio).parameters) == ["pred_corr", "CAD", "PC_aligned", "threshold"]
    assert list(inspect.signature(farthest_point_sample).parameters)[:2] == ["xyz", "ratio"]
