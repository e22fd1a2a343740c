"""(f3) On-disk formats (dpfm_amd/dataset/formats.py), CPU only.

  * BOP scene directory round trip: the LM sample frame (tests/golden/lm_frame.npz: the
    reference's depth PNG, 15 mask_visib PNGs, cam_K) written as a BOP tree (depth PNG, JSONs,
    masks), read back by BopScenes: arrays and JSON entries identical; mapping_list with the
    reference's visib / obj_take filters; object frames -> the oracle crop identical to the one
    built from the golden arrays directly.
  * PLY: ASCII (VCGLIB-style, faces + extra vertex properties) and binary round trips; the
    reference's own models/obj_000001.ply when /root/reference is present (CPU suite only).
  * operator caches: sparse COO L / gradX / gradY as *_idx / *_val, allow_pickle=False, object
    entries refused (not unpickled).
  * result bundles: eval.py's (CAD, PC, Obj) tuple through torch.load(weights_only=True) and
    test_RANSAC.py's field extraction.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import dpfm_oracle as O
from dpfm_amd.dataset import formats as FMT

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _write_bop(root, g, poses):
    from PIL import Image
    scene = root / "train_pbr" / "000000"
    for d in ("depth", "mask_visib", "rgb"):
        (scene / d).mkdir(parents=True, exist_ok=True)
    Image.fromarray(g["depth"].astype(np.uint16)).save(scene / "depth" / "000000.png")
    for j in range(g["masks"].shape[0]):
        Image.fromarray(g["masks"][j].astype(np.uint8)).save(scene / "mask_visib" / f"000000_{j:06d}.png")
    K = g["K"].reshape(-1).tolist()
    (scene / "scene_camera.json").write_text(json.dumps({"0": {"cam_K": K, "depth_scale": float(g["depth_scale"])}}))
    gt, info = [], []
    for j, (R, t, oid) in enumerate(poses):
        gt.append({"cam_R_m2c": R.reshape(-1).tolist(), "cam_t_m2c": (t * 10).tolist(), "obj_id": oid})
        info.append({"visib_fract": float((g["masks"][j] == 255).mean() * 50)})
    (scene / "scene_gt.json").write_text(json.dumps({"0": gt}))
    (scene / "scene_gt_info.json").write_text(json.dumps({"0": info}))
    models = root / "models"
    models.mkdir(exist_ok=True)
    return scene, models


def test_bop_round_trip_and_object_frames(tmp_path):
    from dpfm_amd.dataset.synthetic import random_rotation
    g = np.load(os.path.join(GOLD, "lm_frame.npz"))
    rng = np.random.default_rng(0)
    nobj = g["masks"].shape[0]
    poses = [(random_rotation(rng), rng.normal(size=3) * 5 + np.array([0, 0, 80.0]), 1 + (j % 3)) for j in range(nobj)]
    scene, models = _write_bop(tmp_path, g, poses)
    cads = {oid: rng.normal(size=(200 + oid, 3)) * 40 for oid in (1, 2, 3)}
    for oid, v in cads.items():
        FMT.write_ply(models / f"obj_{oid:06d}.ply", v)
    (models / "models_info.json").write_text(json.dumps({str(o): {"diameter": 100.0 + o} for o in cads}))

    sc = FMT.BopScenes(tmp_path, "train_pbr")
    assert len(sc) == 1
    item = sc[0]
    np.testing.assert_array_equal(item["depth"], g["depth"])
    assert len(item["seg"]) == nobj
    for j in range(nobj):
        np.testing.assert_array_equal(item["seg"][j], g["masks"][j])
    assert item["camera"]["depth_scale"] == float(g["depth_scale"])

    # mapping list: the reference's filters (visib >= min_vis; obj_take when > 1 id)
    info = json.loads((scene / "scene_gt_info.json").read_text())["0"]
    vis = np.array([o["visib_fract"] for o in info])
    m = FMT.collect_mapping_list(sc, min_vis=0.1)
    assert m.tolist() == [[0, j] for j in range(nobj) if vis[j] >= 0.1]
    m2 = FMT.collect_mapping_list(sc, min_vis=0.0, obj_take=(1, 2))
    assert m2.tolist() == [[0, j] for j in range(nobj) if poses[j][2] in (1, 2)]
    FMT.save_mapping_list(tmp_path / "mapping_list.npz", m)
    np.testing.assert_array_equal(FMT.load_mapping_list(tmp_path / "mapping_list.npz"), m)

    # object frame -> the crop the reference forms (object.py:133-148, 174) equals the one from
    # the golden arrays directly
    cache = {}
    for j in (0, 3, 7):
        fr = FMT.object_frame(sc, 0, j, models, cad_cache=cache)
        pts = O.dpt_2_pcld(fr["depth"], 1000 / fr["depth_scale"], fr["K"], fr["mask"] == 255)
        ref = O.dpt_2_pcld(g["depth"], 1000 / float(g["depth_scale"]), g["K"], g["masks"][j] == 255)
        np.testing.assert_array_equal(pts, ref)
        R, t, oid = poses[j]
        np.testing.assert_allclose(fr["R_m2c"], R, rtol=0, atol=1e-15)
        np.testing.assert_allclose(fr["t_m2c"], t, rtol=1e-14)
        np.testing.assert_allclose(fr["cad"], cads[oid] * 0.1, rtol=0, atol=1e-12)
        assert fr["diam_cad"] == pytest.approx((100.0 + oid) * 0.1)


def test_ply_ascii_and_binary(tmp_path):
    rng = np.random.default_rng(1)
    v = rng.normal(size=(37, 3))
    f = rng.integers(0, 37, size=(20, 3))
    FMT.write_ply(tmp_path / "b.ply", v, f)
    p = FMT.read_ply(tmp_path / "b.ply")
    np.testing.assert_array_equal(p.vertices, v)
    np.testing.assert_array_equal(p.faces, f)
    lines = ["ply", "format ascii 1.0", "comment VCGLIB generated", "element vertex 37", "property float x",
             "property float y", "property float z", "property float nx", "property float ny", "property float nz",
             "property uchar red", "property uchar green", "property uchar blue", "property uchar alpha",
             "element face 20", "property list uchar int vertex_indices", "end_header"]
    v32 = v.astype(np.float32)
    for i in range(37):
        lines.append(" ".join(repr(float(x)) for x in v32[i]) + " 0 0 1 255 128 0 255")
    for r in f:
        lines.append("3 " + " ".join(str(int(x)) for x in r))
    (tmp_path / "a.ply").write_text("\n".join(lines) + "\n")
    a = FMT.read_ply(tmp_path / "a.ply")
    np.testing.assert_array_equal(a.vertices, v32.astype(np.float64))
    np.testing.assert_array_equal(a.faces, f)
    assert a.properties["red"][0] == 255


@pytest.mark.skipif(not os.path.exists("/root/reference/sample-data/lm/models/obj_000001.ply"),
                    reason="reference sample data absent")
def test_ply_reads_reference_model():
    p = FMT.read_ply("/root/reference/sample-data/lm/models/obj_000001.ply")
    assert p.vertices.shape == (5841, 3) and p.faces.shape == (11678, 3)
    assert p.faces.min() >= 0 and p.faces.max() < 5841
    info = FMT.load_models_info("/root/reference/sample-data/lm/models")
    d = np.sqrt(((p.vertices[:, None, :] - p.vertices[None, ::7, :]) ** 2).sum(-1)).max()
    assert d <= info["1"]["diameter"] * (1 + 1e-3)


def test_operator_cache_round_trip_and_pickle_refusal(tmp_path):
    rng = np.random.default_rng(2)
    V = 50
    L = torch.sparse_coo_tensor(torch.from_numpy(rng.integers(0, V, size=(2, 200))), torch.randn(200), (V, V)).coalesce()
    ops = {"xyz": torch.randn(V, 3), "mass": torch.rand(V), "evals": torch.rand(64), "evecs": torch.randn(V, 64),
           "frames": torch.randn(V, 3, 3), "L": L, "gradX": L * 2, "gradY": L * 3}
    FMT.save_operator_npz(tmp_path / "CAD_LBO_1.npz", ops)
    z = np.load(tmp_path / "CAD_LBO_1.npz", allow_pickle=False)
    assert {"L_idx", "L_val", "gradX_idx", "gradY_val"} <= set(z.files) and "L" not in z.files
    got = FMT.load_operator_npz(tmp_path / "CAD_LBO_1.npz")
    assert got.refused == []
    for k in ("xyz", "mass", "evals", "evecs", "frames"):
        assert torch.equal(got.data[k], ops[k])
    for k in ("L", "gradX", "gradY"):
        assert torch.equal(got.data[k].to_dense(), ops[k].to_dense())
    # an obj.npz like the reference's: a Path stored as an object array must not be unpickled
    np.savez(tmp_path / "0_0_obj.npz", R_m2c=np.eye(3), cad_path=np.array(object(), dtype=object))
    got = FMT.load_operator_npz(tmp_path / "0_0_obj.npz")
    assert got.refused == ["cad_path"] and torch.equal(got.data["R_m2c"], torch.eye(3, dtype=torch.float64))


def test_result_bundle_round_trip(tmp_path):
    rng = np.random.default_rng(3)
    CAD = {"xyz": torch.randn(500, 3), "evecs": torch.randn(500, 64), "L": None}
    PC = {"xyz": torch.randn(300, 3)}
    Obj = {"P": rng.integers(0, 300, size=(900, 2)), "pcd_depth": rng.normal(size=(300, 3)),
           "R_m2c": np.eye(3), "t_m2c": np.array([1.0, 2.0, 90.0]), "diam_cad": np.float64(12.5),
           "obj_id": np.int64(6), "cad_path": FMT.Path("/data/obj_000006.ply"),
           "p_pred": torch.stack([torch.randint(0, 500, (300,)), torch.arange(300)]),
           "C_pred": torch.randn(30, 30), "ir": torch.tensor(0.42)}
    paths = FMT.write_bundles(tmp_path, [(CAD, PC, Obj)], start_index=7)
    assert [os.path.basename(p) for p in paths] == ["7_obj_6.pt"]
    b = FMT.load_result_bundle(paths[0])
    r = FMT.ransac_inputs(b)
    np.testing.assert_array_equal(r["P_pred"], Obj["p_pred"].numpy().T)
    np.testing.assert_array_equal(r["PC_ver"], Obj["pcd_depth"])
    np.testing.assert_array_equal(r["CAD_ver"], CAD["xyz"].numpy())
    assert r["obj_id"] == 6 and r["diam_cad"] == 12.5 and abs(r["ir"] - 0.42) < 1e-7
    assert FMT.list_bundles(tmp_path) == paths
