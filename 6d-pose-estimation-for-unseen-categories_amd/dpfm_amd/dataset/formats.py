"""On-disk formats of the reference — the (f3) row of SURVEY.md §8(f): read what the reference's
caches and datasets hold, write what its scripts read, without executing anything from a file.

  BOP scene directories      dataset/scene.py:61-158 (`base_scene_dataset`): per frame the depth
                             PNG (uint16), scene_camera.json (cam_K, depth_scale),
                             scene_gt.json (cam_R_m2c, cam_t_m2c in mm, obj_id),
                             scene_gt_info.json (visib_fract), mask_visib/<frame>_<obj>.png and
                             optionally rgb/<frame>.jpg. The reference caches the path lists as
                             a pickle (scene.py:65-74); that cache is not read here (pickles
                             execute code) — `BopScenes` re-globs, which is cheap.
  mapping_list.npz           dataset/object.py:91-115: (scene, object) pairs with visib_fract
                             >= min_vis, filtered by obj_take.
  object frames              dataset/object.py:125-164: the per-object fields the crop path
                             needs (depth, mask == 255, K, depth_scale, R_m2c, t_m2c * 0.1,
                             CAD vertices * 0.1, diameter * 0.1) as the dicts
                             `pipeline.frame_batch` packs into HBM.
  PLY                        models/obj_*.ply (ASCII, VCGLIB) and the results' ply outputs
                             (binary little-endian, Open3D): vertices (+ faces).
  operator caches (npz)      dataset/object.py:240-262, 318-338: CAD_LBO / pc_LBO dicts, sparse
                             L / gradX / gradY stored as `<key>_idx` / `<key>_val` COO parts.
                             Loaded with allow_pickle=False: an object-array entry (the
                             reference's obj.npz stores `cad_path` as a pickled Path) is
                             refused and reported, never unpickled.
  result bundles (.pt)       scripts/eval.py:110-119 writes torch.save((CAD, PC, Obj)) per crop
                             with p_pred / C_pred / ir added to Obj; scripts/test_RANSAC.py:
                             360-378 reads them. Written here with tensors and plain Python
                             values only, so torch.load(weights_only=True) reads them back.
"""
from __future__ import annotations

import functools
import json
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional, Sequence

import numpy as np
import torch

SPARSE_KEYS = ("L", "gradX", "gradY")


# --------------------------------------------------------------------------------------- PLY

_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
              "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


@dataclass
class PlyData:
    vertices: np.ndarray                      # f64 [N, 3]
    faces: Optional[np.ndarray] = None        # int64 [M, 3] (triangles) or None
    properties: dict = field(default_factory=dict)  # every vertex property by name


def _parse_header(f):
    lines = []
    while True:
        line = f.readline()
        if not line:
            raise ValueError("PLY: unexpected end of header")
        line = line.decode("ascii", "replace").strip()
        lines.append(line)
        if line == "end_header":
            break
    if lines[0] != "ply":
        raise ValueError("not a PLY file")
    fmt = next(l.split()[1] for l in lines if l.startswith("format"))
    elements = []
    for l in lines:
        tok = l.split()
        if not tok:
            continue
        if tok[0] == "element":
            elements.append({"name": tok[1], "count": int(tok[2]), "props": []})
        elif tok[0] == "property":
            if tok[1] == "list":
                elements[-1]["props"].append((tok[4], "list", tok[2], tok[3]))
            else:
                elements[-1]["props"].append((tok[2], tok[1]))
    return fmt, elements


def read_ply(path) -> PlyData:
    """Vertices (x, y, z as f64) and triangle faces of an ASCII or binary little-endian PLY."""
    with open(path, "rb") as f:
        fmt, elements = _parse_header(f)
        body = f.read()
    props, verts, faces = {}, None, None
    if fmt == "ascii":
        toks = body.split()
        pos = 0
        for el in elements:
            if el["name"] == "vertex" and all(p[1] != "list" for p in el["props"]):
                k = len(el["props"])
                arr = np.array(toks[pos:pos + k * el["count"]], dtype=np.float64).reshape(el["count"], k)
                pos += k * el["count"]
                for j, p in enumerate(el["props"]):
                    props[p[0]] = arr[:, j]
            else:
                rows = []
                for _ in range(el["count"]):
                    row = []
                    for p in el["props"]:
                        if p[1] == "list":
                            n = int(toks[pos])
                            row.append([int(t) for t in toks[pos + 1:pos + 1 + n]])
                            pos += 1 + n
                        else:
                            row.append(float(toks[pos]))
                            pos += 1
                    rows.append(row)
                if el["name"] == "face":
                    faces = np.array([r[0] for r in rows], dtype=np.int64).reshape(-1, 3) if rows else \
                        np.zeros((0, 3), np.int64)
    elif fmt == "binary_little_endian":
        pos = 0
        for el in elements:
            if all(p[1] != "list" for p in el["props"]):
                dt = np.dtype([(p[0], "<" + _PLY_TYPES[p[1]]) for p in el["props"]])
                arr = np.frombuffer(body, dtype=dt, count=el["count"], offset=pos)
                pos += dt.itemsize * el["count"]
                if el["name"] == "vertex":
                    for p in el["props"]:
                        props[p[0]] = arr[p[0]].astype(np.float64)
            else:
                if len(el["props"]) != 1:
                    raise ValueError("PLY: only single-list face elements are supported")
                _, _, ct, it = el["props"][0]
                cdt, idt = np.dtype("<" + _PLY_TYPES[ct]), np.dtype("<" + _PLY_TYPES[it])
                out = []
                for _ in range(el["count"]):
                    n = int(np.frombuffer(body, dtype=cdt, count=1, offset=pos)[0])
                    pos += cdt.itemsize
                    out.append(np.frombuffer(body, dtype=idt, count=n, offset=pos))
                    pos += idt.itemsize * n
                if el["name"] == "face":
                    faces = np.array(out, dtype=np.int64).reshape(-1, 3) if out else np.zeros((0, 3), np.int64)
    else:
        raise ValueError(f"PLY format {fmt!r} not supported")
    verts = np.stack([props["x"], props["y"], props["z"]], 1)
    return PlyData(vertices=verts, faces=faces, properties=props)


def write_ply(path, vertices: np.ndarray, faces: Optional[np.ndarray] = None) -> None:
    """Binary little-endian PLY with double x / y / z (Open3D's point-cloud output format, as the
    reference's results_poses_RANSAC/ply files are) and optional int triangle faces."""
    v = np.ascontiguousarray(np.asarray(vertices, dtype="<f8").reshape(-1, 3))
    head = ["ply", "format binary_little_endian 1.0", f"element vertex {v.shape[0]}",
            "property double x", "property double y", "property double z"]
    if faces is not None:
        head += [f"element face {len(faces)}", "property list uchar int vertex_indices"]
    head.append("end_header")
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode("ascii"))
        f.write(v.tobytes())
        if faces is not None:
            fc = np.asarray(faces, dtype="<i4").reshape(-1, 3)
            rec = np.zeros(len(fc), dtype=[("n", "u1"), ("i", "<i4", (3,))])
            rec["n"] = 3
            rec["i"] = fc
            f.write(rec.tobytes())


# ------------------------------------------------------------------------------------ BOP

class BopScenes:
    """dataset/scene.py:9-158 `base_scene_dataset` for one BOP dataset split:
    `root` = data_root / render_data_name, `mode` in train / val / test / train_pbr. Item i is the
    reference's dict: depth (uint16 [H, W]), camera / scene_gt / scene_info (the frame's JSON
    entries), seg (list of mask_visib images, uint8), and color when requested. Frames whose
    files are incomplete are dropped, as the reference's check_exists does."""

    def __init__(self, root, mode: str = "train_pbr", color: bool = False, num_samples: int = -1):
        mode = mode.lower()
        if mode == "validation":
            mode = "val"
        if mode not in ("train", "val", "test", "train_pbr"):
            raise ValueError("invalid mode, select train, val, or test")
        self.root, self.mode, self.color = Path(root), mode, color
        self.render_data_name = self.root.name
        self.frames = []
        scanned = 0  # the reference counts every scanned depth path, kept or dropped (scene.py:86-110)
        for depth_path in sorted((self.root / mode).rglob("*/depth/*.png")):
            scene = depth_path.parents[1]
            stem = depth_path.stem
            seg = sorted((scene / "mask_visib").glob(stem + "_*.png"))
            rec = {"depth": depth_path, "camera": scene / "scene_camera.json", "scene_gt": scene / "scene_gt.json",
                   "scene_info": scene / "scene_gt_info.json", "seg": seg}
            if color:
                rec["color"] = (scene / "rgb" / stem).with_suffix(".jpg")
            if all(p.exists() for k, p in rec.items() if k != "seg") and all(p.exists() for p in seg):
                self.frames.append(rec)
            scanned += 1
            if scanned == num_samples:
                break
        self._json = {}

    def __len__(self):
        return len(self.frames)

    def _entry(self, path: Path, key: str):
        if path not in self._json:
            with open(path) as f:
                self._json[path] = json.load(f)
        return self._json[path][key]

    def __getitem__(self, idx: int) -> dict:
        from PIL import Image
        rec = self.frames[idx]
        sub = str(int(rec["depth"].stem))
        out = {"depth": np.asarray(Image.open(rec["depth"])),
               "camera": self._entry(rec["camera"], sub),
               "scene_gt": self._entry(rec["scene_gt"], sub),
               "scene_info": self._entry(rec["scene_info"], sub),
               "seg": [np.asarray(Image.open(p)) for p in rec["seg"]],
               "scene_nr": None, "subscene_nr": None}
        if self.color:
            out["color"] = np.asarray(Image.open(rec["color"]))
        return out


def collect_mapping_list(scenes: BopScenes, min_vis: float = 0.0, obj_take: Sequence[int] = ()) -> np.ndarray:
    """dataset/object.py:101-110: int64 [M, 2] (frame i, object j) with visib_fract >= min_vis
    and, when obj_take lists more than one id, obj_id in obj_take (the reference's filter)."""
    out = []
    for i in range(len(scenes)):
        rec = scenes.frames[i]
        sub = str(int(rec["depth"].stem))
        info = scenes._entry(rec["scene_info"], sub)
        gt = scenes._entry(rec["scene_gt"], sub)
        for j, obj in enumerate(info):
            if obj["visib_fract"] < min_vis:
                continue
            if len(obj_take) > 1 and gt[j]["obj_id"] not in obj_take:
                continue
            out.append((i, j))
    return np.asarray(out, dtype=np.int64).reshape(-1, 2)


def save_mapping_list(path, mapping: np.ndarray) -> None:
    np.savez(path, mapping_list=np.asarray(mapping, dtype=np.int64))


def load_mapping_list(path) -> np.ndarray:
    with np.load(path, allow_pickle=False) as z:
        return np.asarray(z["mapping_list"], dtype=np.int64).reshape(-1, 2)


def load_models_info(models_dir) -> dict:
    return dict(_models_info(str(Path(models_dir).resolve())))


@functools.lru_cache(maxsize=16)
def _models_info(models_dir: str) -> dict:
    with open(Path(models_dir) / "models_info.json") as f:
        return json.load(f)


_CAD_CACHE: dict = {}  # (models_dir, obj_id) -> vertices * 0.1: a PLY is parsed once per process


def object_frame(scenes: BopScenes, i: int, j: int, models_dir, cad_cache: Optional[dict] = None) -> dict:
    """The fields dataset/object.py:133-164 derives for (frame i, object j), as the dict
    `pipeline.frame_batch` packs: depth, mask (mask_visib == 255 test done by the crop kernels
    on value 255), K, depth_scale, R_m2c, t_m2c (* 0.1: cm), cad (model vertices * 0.1 —
    the reference decimates the mesh to 10k faces with Open3D first, :199; out of scope here,
    pass a decimated vertex set through `cad_cache` to reproduce it), diam_cad (* 0.1)."""
    sc = scenes[i]
    gt = sc["scene_gt"][j]
    oid = int(gt["obj_id"])
    models_dir = Path(models_dir)
    if cad_cache is None:  # module-level cache keyed by the models directory
        key = (str(models_dir.resolve()), oid)
        if key not in _CAD_CACHE:
            _CAD_CACHE[key] = read_ply(models_dir / f"obj_{oid:06d}.ply").vertices * 0.1
        cad = _CAD_CACHE[key]
    else:
        if oid not in cad_cache:
            cad_cache[oid] = read_ply(models_dir / f"obj_{oid:06d}.ply").vertices * 0.1
        cad = cad_cache[oid]
    info = _models_info(str(models_dir.resolve()))
    return {"depth": sc["depth"], "mask": sc["seg"][j], "K": np.asarray(sc["camera"]["cam_K"], np.float64).reshape(3, 3),
            "depth_scale": float(sc["camera"]["depth_scale"]),
            "R_m2c": np.asarray(gt["cam_R_m2c"], np.float64).reshape(3, 3),
            "t_m2c": np.asarray(gt["cam_t_m2c"], np.float64) * 0.1, "obj_id": oid,
            "visib_fract": float(sc["scene_info"][j]["visib_fract"]),
            "cad": cad, "diam_cad": float(info[str(oid)]["diameter"]) * 0.1,
            "rgb": sc.get("color")}


# --------------------------------------------------------------------------- operator caches

def save_operator_npz(path, ops: dict, sparse_keys: Sequence[str] = SPARSE_KEYS) -> None:
    """dataset/object.py:240-262 + save_sparse_tensor (:318-325): dense entries as arrays, each
    sparse COO operator as `<key>_idx` (int64 [2, nnz]) and `<key>_val`."""
    out = {}
    for k, v in ops.items():
        if k in sparse_keys and v is not None:
            v = v.coalesce() if isinstance(v, torch.Tensor) else torch.as_tensor(v).to_sparse().coalesce()
            out[k + "_idx"] = v.indices().cpu().numpy()
            out[k + "_val"] = v.values().cpu().numpy()
        elif v is not None:
            out[k] = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
    np.savez(path, **out)


@dataclass
class LoadedNpz:
    data: dict
    refused: list  # keys whose entries need unpickling (object arrays): not loaded


def load_operator_npz(path, sparse_keys: Sequence[str] = SPARSE_KEYS, to_tensor: bool = True) -> LoadedNpz:
    """dict(np.load(path)) + dict_to_tensor (object.py:326-338) with allow_pickle=False: sparse
    keys become torch.sparse_coo_tensor of shape [V, V] (V = evecs rows); dense arrays become
    tensors when to_tensor. Object-array entries are refused (listed in `.refused`)."""
    data, refused = {}, []
    with np.load(path, allow_pickle=False) as z:
        for k in z.files:
            try:
                data[k] = z[k]
            except ValueError:  # object array: would need pickle
                refused.append(k)
    if "evecs" in data:
        V = data["evecs"].shape[0]
        for key in sparse_keys:
            if key + "_idx" in data and key + "_val" in data:
                idx, val = data.pop(key + "_idx"), data.pop(key + "_val")
                data[key] = torch.sparse_coo_tensor(torch.as_tensor(idx), torch.as_tensor(val), (V, V))
    if to_tensor:
        data = {k: (torch.as_tensor(v) if isinstance(v, np.ndarray) and v.dtype != np.dtype("U") and
                    v.dtype.kind in "biuf" else v) for k, v in data.items()}
    return LoadedNpz(data, refused)


# ---------------------------------------------------------------------------- result bundles

def _plain(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu()
    if isinstance(v, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(v)) if v.dtype.kind in "biuf" else v.tolist()
    if isinstance(v, (np.floating, np.integer)):
        return v.item()
    if isinstance(v, Path):
        return str(v)
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return type(v)(_plain(x) for x in v)
    return v


def save_result_bundle(path, CAD: dict, PC: dict, Obj: dict) -> None:
    """scripts/eval.py:110-119: torch.save((CAD, PC, Obj)) for one crop, Obj carrying p_pred
    ([2, n] int64: CAD index row, PC index row), C_pred and ir. Tensors and plain values only."""
    torch.save((_plain(CAD), _plain(PC), _plain(Obj)), path)


def load_result_bundle(path):
    """The (CAD, PC, Obj) tuple, read with torch.load(weights_only=True) (no code runs)."""
    return torch.load(path, map_location="cpu", weights_only=True)


def ransac_inputs(bundle) -> dict:
    """What scripts/test_RANSAC.py:366-378 takes out of a bundle: P_gt, P_pred ([n, 2] = p_pred.T),
    CAD_ver, PC_ver (pcd_depth), R_m2c, t_m2c, diam_cad, ir, obj_id — as numpy."""
    cad, _, obj = bundle
    npy = lambda v: v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)  # noqa: E731
    return {"P_gt": npy(obj["P"]), "P_pred": npy(obj["p_pred"]).T, "CAD_ver": npy(cad["xyz"]),
            "PC_ver": npy(obj["pcd_depth"]), "R_m2c": npy(obj["R_m2c"]), "t_m2c": npy(obj["t_m2c"]),
            "diam_cad": float(npy(obj["diam_cad"])), "ir": float(npy(obj["ir"])), "obj_id": int(npy(obj["obj_id"]))}


def write_bundles(out_dir, crops: Sequence[tuple], start_index: int = 0) -> list:
    """eval.py's naming: f"{idx}_obj_{obj_id}.pt" per crop, idx counting from start_index."""
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for k, (CAD, PC, Obj) in enumerate(crops):
        p = os.path.join(out_dir, f"{start_index + k}_obj_{int(_plain(Obj['obj_id']))}.pt")
        save_result_bundle(p, CAD, PC, Obj)
        paths.append(p)
    return paths


def list_bundles(directory) -> list:
    """test_RANSAC.py:335-342: the .pt files of a results directory in sorted order."""
    return [os.path.join(directory, f) for f in sorted(os.listdir(directory)) if f.endswith(".pt")]

