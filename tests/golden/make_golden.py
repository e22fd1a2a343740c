"""Mint tests/golden fixtures from data files the reference itself holds.

Run in the development container (needs /root/reference, read-only):
    python tests/golden/make_golden.py
Nothing here imports or runs reference code; it reads PNG / JSON / PLY / TXT data:

  lm_frame.npz   sample-data/lm/train_pbr/000000: depth png, every mask_visib png,
                 cam_K + depth_scale of scene_camera.json (H1/H2/H3 real-data inputs)
  pose_metrics.npz  H14 golden vectors: for N published crops of
                 results_on_{pbr,real}/results_poses_RANSAC, the CAD vertices
                 (ply/…/cad_i.ply), T_gt and T_pred_ICP recovered at full precision from
                 cad_i_pose_gt.ply / cad_i_pose_est.ply (the reference wrote those plys as
                 CAD transformed by the full-precision poses), T_pred as printed, and the
                 reference's printed metrics (ADD ICP, Add Score ICP thres (xyz direction),
                 Add-S Score ICP, Error [cm], Error [deg], diameter from models_info.json)
  p_pred.npy     sample-data/sample_P_pred/p_i0.npy (RANSAC correspondence shape/order)
  real_crops.npz 7 published crops + the 5 decimated CADs (see real_crops)
  icp_pin.npz    512 published crops: T_gt, printed T_pred, the reference's ICP output (see icp_pin)
"""
import glob
import json
import os
import re

import numpy as np
from PIL import Image

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def read_ply_xyz(path):
    with open(path, "rb") as f:
        header = b""
        while not header.endswith(b"end_header\n"):
            header += f.readline()
        h = header.decode()
        n = int(re.search(r"element vertex (\d+)", h).group(1))
        props = re.findall(r"property (\w+) (\w+)", h.split("element vertex")[1].split("element")[0])
        assert "binary_little_endian" in h
        dt = {"double": "<f8", "float": "<f4"}
        dtype = np.dtype([(name, dt[t]) for t, name in props])
        data = np.frombuffer(f.read(n * dtype.itemsize), dtype=dtype, count=n)
    return np.stack([data["x"], data["y"], data["z"]], 1).astype(np.float64)


def parse_result_txt(path):
    txt = open(path).read()

    def num(label):
        m = re.search(re.escape(label) + r":\s*([-+0-9.eEnaif]+)", txt)
        return float(m.group(1))

    def mat(label):
        m = re.search(re.escape(label) + r".*?\n(\[\[.*?\]\])", txt, re.S)
        return np.array([[float(x) for x in row.replace("[", "").replace("]", "").split()]
                         for row in m.group(1).strip().split("\n")])

    return dict(obj_id=int(num("Object ID")), add=num("Avg. Euclidean Distance (ADD) [cm]"),
                add_icp=num("Avg. Euclidean Distance (ADD) ICP"),
                add_xyz_icp=num("Add Score ICP thres (xyz direction)"),
                adds_icp=num("Add-S Score ICP"), err_cm=num("Error [cm]"), err_deg=num("Error [deg]"),
                T_gt=mat("T_gt (Ground Truth Transformation):"),
                T_pred=mat("T_pred (Predicted Transformation):"),
                T_icp=mat("T_pred_ICP (Predicted Transformation from ICP):"))


def fit_rigid(src, dst):
    """Least-squares [R|t] with dst = src @ R.T + t (exact data -> exact up to rounding)."""
    A = np.concatenate([src, np.ones((src.shape[0], 1))], 1)
    X, *_ = np.linalg.lstsq(A, dst, rcond=None)
    T = np.eye(4)
    T[:3, :3] = X[:3].T
    T[:3, 3] = X[3]
    return T


def main():
    base = f"{REF}/sample-data/lm/train_pbr/000000"
    depth = np.asarray(Image.open(f"{base}/depth/000000.png"))
    masks = np.stack([np.asarray(Image.open(p)) for p in sorted(glob.glob(f"{base}/mask_visib/000000_*.png"))])
    cam = json.load(open(f"{base}/scene_camera.json"))["0"]
    np.savez_compressed(f"{OUT}/lm_frame.npz", depth=depth, masks=masks,
                        K=np.array(cam["cam_K"], dtype=np.float64).reshape(3, 3),
                        depth_scale=np.float64(cam["depth_scale"]))

    info = json.load(open(f"{REF}/sample-data/lm/models/models_info.json"))
    rows = []
    for tree in ("results_on_pbr", "results_on_real"):
        files = sorted(glob.glob(f"{REF}/{tree}/results_poses_RANSAC/results/*.txt"))
        for path in files[:4]:
            name = os.path.basename(path)[:-4]
            i = name.split("_")[-1]
            d = f"{REF}/{tree}/results_poses_RANSAC/ply/{name}"
            if not os.path.exists(f"{d}/cad_{i}.ply"):
                continue
            r = parse_result_txt(path)
            cad = read_ply_xyz(f"{d}/cad_{i}.ply")
            T_gt = fit_rigid(cad, read_ply_xyz(f"{d}/cad_{i}_pose_gt.ply"))
            T_icp = fit_rigid(cad, read_ply_xyz(f"{d}/cad_{i}_pose_est.ply"))
            assert np.allclose(T_gt, r["T_gt"], atol=1e-6), name
            assert np.allclose(T_icp, r["T_icp"], atol=1e-6), name
            r.update(cad=cad, T_gt_full=T_gt, T_icp_full=T_icp,
                     diam=info[str(r["obj_id"])]["diameter"] * 0.1, tree=tree, name=name)
            rows.append(r)
    out = {}
    for k, r in enumerate(rows):
        for key in ("cad", "T_gt_full", "T_icp_full", "T_pred", "add", "add_icp", "add_xyz_icp", "adds_icp",
                    "err_cm", "err_deg", "diam", "obj_id"):
            out[f"{k}_{key}"] = np.asarray(r[key])
    out["n"] = np.int64(len(rows))
    np.savez_compressed(f"{OUT}/pose_metrics.npz", **out)
    np.save(f"{OUT}/p_pred.npy", np.load(f"{REF}/sample-data/sample_P_pred/p_i0.npy"))
    cads = real_crops(info)
    n_icp = icp_pin(cads)
    print(f"wrote lm_frame.npz, pose_metrics.npz ({len(rows)} crops), p_pred.npy, real_crops.npz, "
          f"icp_pin.npz ({n_icp} crops)")


# Real crops of the published PBR/RANSAC results, chosen to span the reference's crop sizes:
# 200 .. 2000 points (1999 = the int(2000/n * n) rounding of object.py:145-147) on decimated
# CADs of 4996 / 4998 / 5002 vertices (object.py:171-173).
REAL_CROPS = ("obj_11_result_263", "obj_6_result_101", "obj_6_result_409", "obj_5_result_249",
              "obj_11_result_5", "obj_12_result_111", "obj_8_result_196")


def real_crops(info):
    """real_crops.npz: per crop the camera-frame crop pc_i.ply (pcd_depth, f64 cm), T_gt at
    full precision (fitted from cad_i -> cad_i_pose_gt, checked against the printed matrix),
    the object's diameter (models_info.json * 0.1) and id; one decimated CAD per object."""
    base = f"{REF}/results_on_pbr/results_poses_RANSAC"
    out, cads = {}, {}
    for k, name in enumerate(REAL_CROPS):
        i = name.split("_")[-1]
        d = f"{base}/ply/{name}"
        r = parse_result_txt(f"{base}/results/{name}.txt")
        cad = read_ply_xyz(f"{d}/cad_{i}.ply")
        T_gt = fit_rigid(cad, read_ply_xyz(f"{d}/cad_{i}_pose_gt.ply"))
        assert np.allclose(T_gt, r["T_gt"], atol=1e-6), name
        oid = r["obj_id"]
        if oid in cads:
            assert np.array_equal(cads[oid], cad), name  # one decimated CAD per object
        cads[oid] = cad
        out[f"{k}_pc"] = read_ply_xyz(f"{d}/pc_{i}.ply")
        out[f"{k}_T_gt"] = T_gt
        out[f"{k}_obj_id"] = np.int64(oid)
        out[f"{k}_diam"] = np.float64(info[str(oid)]["diameter"] * 0.1)
        out[f"{k}_n_corr"] = np.int64(int(re.search(r"Num\. of correspondences:\s*(\d+)",
                                                    open(f"{base}/results/{name}.txt").read()).group(1)))
    for oid, cad in cads.items():
        out[f"cad_{oid}"] = cad
    out["n"] = np.int64(len(REAL_CROPS))
    np.savez_compressed(f"{OUT}/real_crops.npz", **out)
    return cads


TREES = ("results_on_pbr", "results_on_real")
SOLVERS = ("RANSAC", "TEASER")


def icp_pin(cads, per_dir=128):
    """icp_pin.npz: the reference's own Open3D ICP outputs (f4 / Umeyama pin).

    test_RANSAC.py:424-446 (test_teaser.py:469-483 likewise) refines the solver's T_est with
    registration_icp(source = CAD, target = transform(CAD, T_gt), r = 0.2, init = T_est,
    PointToPoint, max_iteration = 2000) and stores, per crop, cad_i.ply, cad_i_pose_gt.ply
    (= the target), cad_i_pose_est.ply (= CAD under the ICP result) and the txt with T_pred
    printed to 9 digits. Per crop this keeps: the object id (CAD = real_crops.npz cad_<id>,
    checked identical here), T_gt and T_icp fitted at full precision from the plys (checked
    against the printed matrices), T_pred as printed (the ICP init). per_dir crops are taken
    evenly strided from each of the four result directories (sorted file order)."""
    rows = {k: [] for k in ("obj_id", "tree", "solver", "index", "T_gt", "T_pred", "T_icp", "target_dev")}
    for ti, tree in enumerate(TREES):
        for si, solver in enumerate(SOLVERS):
            base = f"{REF}/{tree}/results_poses_{solver}"
            files = sorted(glob.glob(f"{base}/results/*.txt"))
            pick = np.unique(np.linspace(0, len(files) - 1, per_dir).round().astype(int))
            for k in pick:
                name = os.path.basename(files[k])[:-4]
                i = name.split("_")[-1]
                d = f"{base}/ply/{name}"
                r = parse_result_txt(files[k])
                cad = read_ply_xyz(f"{d}/cad_{i}.ply")
                assert np.array_equal(cad, cads[r["obj_id"]]), name
                tgt = read_ply_xyz(f"{d}/cad_{i}_pose_gt.ply")
                T_gt = fit_rigid(cad, tgt)
                T_icp = fit_rigid(cad, read_ply_xyz(f"{d}/cad_{i}_pose_est.ply"))
                assert np.allclose(T_gt, r["T_gt"], atol=1e-6), name
                assert np.allclose(T_icp, r["T_icp"], atol=1e-6), name
                # the test rebuilds the target as transform(CAD, T_gt) (test_RANSAC.py:154-160)
                dev = np.abs(cad @ T_gt[:3, :3].T + T_gt[:3, 3] - tgt).max()
                for key, v in (("obj_id", r["obj_id"]), ("tree", ti), ("solver", si), ("index", int(i)),
                               ("T_gt", T_gt), ("T_pred", r["T_pred"]), ("T_icp", T_icp), ("target_dev", dev)):
                    rows[key].append(v)
    out = {k: np.asarray(v) for k, v in rows.items()}
    np.savez_compressed(f"{OUT}/icp_pin.npz", **out)
    return len(rows["obj_id"])


if __name__ == "__main__":
    main()
