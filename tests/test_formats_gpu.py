"""(f3) The BOP reader feeding the device crop path: frames written as a BOP tree (the LM sample
frame of tests/golden/lm_frame.npz), read back by formats.BopScenes / object_frame, packed by
pipeline.frame_batch and formed by CropFormation (reference policy npoint = 0): padded crops,
align_pc, overlaps and pair lists bit-exact against the oracle chain per object
(object.py:133-180) followed by the oracle's collate."""
import os

import numpy as np
import pytest
import torch

from oracle import dpfm_oracle as O
from test_formats_cpu import _write_bop, GOLD

pytestmark = pytest.mark.gpu


def test_bop_frames_through_crop_formation(tmp_path, device):
    from dpfm_amd.dataset import formats as FMT
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.dataset.synthetic import random_rotation
    from dpfm_amd.pipeline import frame_batch
    g = np.load(os.path.join(GOLD, "lm_frame.npz"))
    rng = np.random.default_rng(4)
    nobj = g["masks"].shape[0]
    poses = [(random_rotation(rng), rng.normal(size=3) * 3 + np.array([0, 0, 90.0]), 1 + (j % 2)) for j in range(nobj)]
    _, models = _write_bop(tmp_path, g, poses)
    import json
    for oid in (1, 2):
        FMT.write_ply(models / f"obj_{oid:06d}.ply", rng.normal(size=(400 + oid, 3)) * 30)
    (models / "models_info.json").write_text(json.dumps({"1": {"diameter": 120.0}, "2": {"diameter": 90.0}}))
    sc = FMT.BopScenes(tmp_path, "train_pbr")
    mapping = FMT.collect_mapping_list(sc, min_vis=0.0)
    cache = {}
    frames = [FMT.object_frame(sc, int(i), int(j), models, cad_cache=cache) for i, j in mapping]
    seed = 5
    crops = CropFormation(npoint=0, seed=seed, pad="batch")(frame_batch(frames, device))
    items = []
    for b, f in enumerate(frames):
        pcd = O.remove_outliers(O.dpt_2_pcld(f["depth"], 1000 / f["depth_scale"], f["K"], f["mask"] == 255))
        pcd = O.sample_crop(pcd, seed, b, fixed=0)
        align = O.transform(pcd, f["R_m2c"], f["t_m2c"], inv=True)
        P = O.find_positives(f["cad"], align, r=f["diam_cad"] * 0.05)
        o12, o21 = O.get_overlap(f["cad"].shape[0], pcd.shape[0], P)
        items.append(({"xyz": f["cad"]}, {"xyz": pcd.astype(np.float32)},
                      {"align_pc": align, "P": P, "overlap_12": o12, "overlap_21": o21, "obj_id": b}))
    CAD, PC, Obj = O.collate(items)
    assert crops.n2.cpu().tolist() == [it[1]["xyz"].shape[0] for it in items]
    assert torch.equal(crops.pc32.cpu(), PC["xyz"])
    assert torch.equal(crops.align32.cpu(), Obj["align_pc"])
    assert torch.equal(crops.overlap_21.cpu().float(), Obj["overlap_21"])
    npairs = crops.npairs.cpu().numpy()
    pairs = crops.pairs.cpu().numpy()
    for b, P in enumerate(Obj["P"]):
        assert npairs[b] == np.asarray(P).reshape(-1, 2).shape[0], b
        np.testing.assert_array_equal(pairs[b, :npairs[b]], np.asarray(P).reshape(-1, 2).astype(np.int64))
