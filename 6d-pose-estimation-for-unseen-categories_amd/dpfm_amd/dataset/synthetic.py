"""Seeded synthetic RGB-D frames, CAD models and spectral operators.

There is no network and no BOP data on the GPU box, so benchmarks and parity tests
run on frames of the same shape and units as the reference's LM PBR data
(sample-data/lm/train_pbr/000000/scene_camera.json):

  frame   640x480 uint16 depth, depth_scale 0.1 (png unit = 0.1 mm), LM PBR K,
          background plane at 1000 mm, one ray-cast ellipsoid (semi-axes 4.5-7 cm,
          centre z 70-100 cm, uniform SO(3) orientation); mask_visib = silhouette
          (255/0, as the reference reads `seg[j] == 255`); RGB = Lambert shading.
  CAD     n1 surface samples of the same ellipsoid in the object frame, cm
          (diam = 2 * max semi-axis, as models_info.json diameter * 0.1)
  pose    R_m2c, t_m2c (cm) with camera = R @ obj + t (BOP convention, object.py:157-158)
  LBO     mass = area / N, evecs = mass-orthonormal Gaussian [N, 64], evals sorted
          U(0, 2) with evals[0] = 0 (stand-in for the cached get_operators output).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

LM_K = np.array([[572.4114, 0.0, 325.2611082792282],
                 [0.0, 573.57043, 242.04899594187737],
                 [0.0, 0.0, 1.0]])
DEPTH_SCALE = 0.1
H, W = 480, 640


def random_rotation(rng: np.random.Generator) -> np.ndarray:
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


@dataclass
class Frame:
    depth: np.ndarray      # uint16 [H, W]
    rgb: np.ndarray        # uint8 [H, W, 3]
    mask: np.ndarray       # uint8 [H, W] 255 / 0 (mask_visib)
    K: np.ndarray          # f64 [3, 3]
    depth_scale: float
    R_m2c: np.ndarray      # f64 [3, 3]
    t_m2c: np.ndarray      # f64 [3] cm
    axes: np.ndarray       # f64 [3] semi-axes cm
    diam_cad: float        # cm


def make_frame(seed: int, axes_range=(4.5, 7.0), z_range=(70.0, 100.0)) -> Frame:
    rng = np.random.default_rng(seed)
    axes = rng.uniform(*axes_range, size=3)
    R = random_rotation(rng)
    zc = rng.uniform(*z_range)
    # keep the object near the optical axis so the silhouette is fully inside the image
    xc, yc = rng.uniform(-8.0, 8.0), rng.uniform(-6.0, 6.0)
    c = np.array([xc, yc, zc])
    K = LM_K
    v, u = np.indices((H, W))
    d = np.stack([(u - K[0, 2]) / K[0, 0], (v - K[1, 2]) / K[1, 1], np.ones_like(u, dtype=np.float64)], -1)
    Dinv = 1.0 / axes
    e = (d @ R) * Dinv           # D R^T d  (row vectors)
    f = (R.T @ c) * Dinv          # D R^T c
    ee = (e * e).sum(-1)
    ef = e @ f
    ff = f @ f
    disc = ef * ef - ee * (ff - 1.0)
    hit = disc > 0
    z = np.where(hit, (ef - np.sqrt(np.maximum(disc, 0.0))) / ee, np.inf)
    z_bg = 100.0  # cm (1000 mm plane)
    obj = hit & (z < z_bg)
    zcm = np.where(obj, z, z_bg)
    depth = np.round(zcm * 100.0).astype(np.uint16)  # 0.1 mm units
    mask = np.where(obj, 255, 0).astype(np.uint8)
    # Lambert shading of the ellipsoid normal for the RGB image
    p = zcm[..., None] * d
    q = ((p - c) @ R) * Dinv * Dinv
    n = q @ R.T
    n /= np.linalg.norm(n, axis=-1, keepdims=True) + 1e-12
    shade = np.clip(-(n * d / np.linalg.norm(d, axis=-1, keepdims=True)).sum(-1), 0, 1)
    base = rng.uniform(60, 255, size=3)
    rgb = np.where(obj[..., None], shade[..., None] * base, 40.0 + 10.0 * (u[..., None] % 7)).astype(np.uint8)
    return Frame(depth=depth, rgb=rgb, mask=mask, K=K.copy(), depth_scale=DEPTH_SCALE, R_m2c=R, t_m2c=c,
                 axes=axes, diam_cad=float(2.0 * axes.max()))


def cad_points(frame: Frame, n: int, seed: int) -> np.ndarray:
    """n surface samples of the frame's ellipsoid in the object frame (cm), f64 [n, 3]."""
    rng = np.random.default_rng(seed + 1_000_003)
    g = rng.normal(size=(n, 3))
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    return g * frame.axes[None, :]


def lbo_operators(n: int, k: int, seed: int, area: float = 300.0):
    """mass f32 [n], evals f32 [k], evecs f32 [n, k] with evecs^T diag(mass) evecs = I."""
    rng = np.random.default_rng(seed + 2_000_003)
    mass = np.full(n, area / n, dtype=np.float64)
    g = rng.normal(size=(n, k))
    q, _ = np.linalg.qr(g)
    evecs = q / np.sqrt(mass)[:, None]
    evals = np.sort(rng.uniform(0.0, 2.0, size=k))
    evals[0] = 0.0
    return mass.astype(np.float32), evals.astype(np.float32), evecs.astype(np.float32)


def ragged_frames(F: int, seed: int, n1: int = 5000) -> list:
    """Frames at the reference's real sizes (tests/golden/real_crops.npz): objects of
    1.5-7 cm semi-axes at 70-100 cm give masks of a few hundred to ~10k pixels, so the sample
    policy (object.py:145-148) yields crops of ~200-2000 points; CADs of n1 +- 3 vertices (the
    reference's decimated CADs have 4996-5002). Dicts with the fields pipeline.frame_batch reads."""
    rng = np.random.default_rng(seed + 7_000_003)
    out = []
    for f in range(F):
        top = float(rng.uniform(1.5, 7.0))
        fr = make_frame(seed + f, axes_range=(0.75 * top, top))
        n = n1 + int(rng.integers(-4, 3))
        out.append(dict(depth=fr.depth, mask=fr.mask, rgb=fr.rgb, K=fr.K, depth_scale=fr.depth_scale,
                        R_m2c=fr.R_m2c, t_m2c=fr.t_m2c, cad=cad_points(fr, n, seed + f), diam_cad=fr.diam_cad))
    return out

