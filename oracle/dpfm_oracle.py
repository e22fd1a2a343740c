"""Literal CPU restatements of the reference hot path — TEST INFRASTRUCTURE ONLY.

Each function cites the /root/reference file:line it restates. Upstream code from
the un-vendored DPFM submodule and Open3D is restated from their public sources
 and is marked "parity unpinned".

Nothing here is imported by the product package.
"""
from __future__ import annotations

import math

import numpy as np
import torch

# --------------------------------------------------------------------------------------
# H1  crop formation: dataset/object.py:52-88
# --------------------------------------------------------------------------------------


def erode_seg_mask(mask: np.ndarray, kernel_size: int = 3) -> np.ndarray:
    """dataset/object.py:52-71 — cv2.erode(uint8*255, plus-shaped 3x3, iterations=1).

    OpenCV's default border for erosion (BORDER_CONSTANT with
    morphologyDefaultBorderValue) never erodes at the image edge, so pixels outside
    the image are ignored. OpenCV itself is absent here: parity unpinned, exact by
    construction for a binary min filter.
    """
    assert kernel_size == 3
    m = mask.astype(bool)
    out = m.copy()
    out[1:, :] &= m[:-1, :]
    out[:-1, :] &= m[1:, :]
    out[:, 1:] &= m[:, :-1]
    out[:, :-1] &= m[:, 1:]
    return out


def dpt_2_pcld(dpt: np.ndarray, cam_scale: float, K: np.ndarray, mask: np.ndarray) -> np.ndarray:
    """dataset/object.py:73-88 (erosion at :80). Returns f64 [P,3] in cm, row-major pixel order."""
    idx = np.indices(dpt.shape[:2])
    xmap = idx[0]
    ymap = idx[1]
    if len(dpt.shape) > 2:
        dpt = dpt[:, :, 0]
    dpt = dpt.astype(np.float32) / np.float32(cam_scale)
    mask = erode_seg_mask(mask, 3)
    dpt = dpt[mask]
    row = (ymap[mask] - K[0, 2]) * dpt.astype(np.float64) / K[0, 0]
    col = (xmap[mask] - K[1, 2]) * dpt.astype(np.float64) / K[1, 1]
    dpt_3d = np.concatenate((row[..., None], col[..., None], dpt.astype(np.float64)[..., None]), axis=1)
    return dpt_3d * 100


# --------------------------------------------------------------------------------------
# H2  statistical outlier removal: dataset/object.py:33-50 -> Open3D 0.17
#     PointCloud::RemoveStatisticalOutliers(nb_neighbors=20, std_ratio=0.3)
#     (parity unpinned: Open3D absent; restated per SURVEY.md Appendix A)
# --------------------------------------------------------------------------------------


def sor_avg_distances(pcd: np.ndarray, nb_neighbors: int = 20) -> np.ndarray:
    """Per point: mean of sqrt(squared distance) to its nb nearest points (self included),
    squared distances as ((dx²+dy²)+dz²) in fp64, summed in ascending order."""
    n = pcd.shape[0]
    k = min(nb_neighbors, n)
    out = np.empty(n, dtype=np.float64)
    for s in range(0, n, 512):
        d = pcd[s:s + 512, None, :] - pcd[None, :, :]
        sq = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
        part = np.partition(sq, k - 1, axis=1)[:, :k]
        part.sort(axis=1)
        r = np.sqrt(part)
        acc = np.zeros(r.shape[0])
        for c in range(k):  # std::accumulate, left to right
            acc = acc + r[:, c]
        out[s:s + 512] = acc / k
    return out


def remove_outliers_indices(pcd: np.ndarray, nb_neighbors: int = 20, std_ratio: float = 0.3) -> np.ndarray:
    avg = sor_avg_distances(pcd, nb_neighbors)
    valid = avg.shape[0]
    if valid == 0:
        return np.zeros(0, dtype=np.int64)
    mean = 0.0
    for a in avg:  # accumulate, skipping non-positive entries
        if a > 0:
            mean = mean + a
    mean = mean / valid
    sq = 0.0
    for a in avg:
        sq = sq + ((a - mean) * (a - mean) if a > 0 else 0.0)
    std = math.sqrt(sq / (valid - 1)) if valid > 1 else float("nan")
    thr = mean + std_ratio * std
    return np.nonzero((avg > 0) & (avg < thr))[0].astype(np.int64)


def remove_outliers(pcd: np.ndarray) -> np.ndarray:
    """dataset/object.py:33-50."""
    return pcd[remove_outliers_indices(pcd, 20, 0.3)]


# --------------------------------------------------------------------------------------
# H3  farthest point sampling: upstream DPFM dpfm/utils.py::farthest_point_sample,
#     called at dataset/object.py:145-148 (parity unpinned; Appendix A)
# --------------------------------------------------------------------------------------


def farthest_point_sample(xyz: torch.Tensor, ratio: float, start: int, npoint: int | None = None) -> torch.Tensor:
    """Literal torch-CPU restatement. xyz f32 [3, N]; `start` replaces torch.randint(0, N)."""
    xyz = xyz.t().unsqueeze(0)
    B, N, C = xyz.shape
    if npoint is None:
        npoint = int(ratio * N)
    centroids = torch.zeros(B, npoint, dtype=torch.long)
    distance = torch.ones(B, N) * 1e10
    farthest = torch.tensor([start], dtype=torch.long)
    batch_indices = torch.arange(B, dtype=torch.long)
    for i in range(npoint):
        centroids[:, i] = farthest
        centroid = xyz[batch_indices, farthest, :].view(B, 1, 3)
        dist = torch.sum((xyz - centroid) ** 2, -1)
        mask = dist < distance
        distance[mask] = dist[mask]
        farthest = torch.max(distance, -1)[1]
    return centroids[0]


def fps_npoint(n: int) -> int:
    """dataset/object.py:145-147: ratio = 2000/N, npoint = int(ratio * N) (1999 or 2000)."""
    ratio = 2000 / n
    return int(ratio * n)


_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def fps_start(seed: int, b: int, n: int) -> int:
    """The FPS start index that replaces upstream's unseeded torch.randint(0, N) for crop b
    (the build's documented choice, include/posekern.h pk_fps_npoint)."""
    return _splitmix64((seed & _M64) ^ _splitmix64(b)) % n if n > 0 else 0


def sample_crop(pcd: np.ndarray, seed: int, b: int, fixed: int = 0, limit: int = 2000) -> np.ndarray:
    """dataset/object.py:145-148 on one outlier-filtered crop: FPS when the crop has more
    than `limit` points (npoint = int(limit/n * n)), every point otherwise. fixed > 0 is the
    build's fixed-size variant (FPS to exactly `fixed` when larger, every point otherwise)."""
    n = pcd.shape[0]
    if fixed > 0:
        npoint = fixed if n > fixed else 0
    else:
        npoint = int(limit / n * n) if n > limit else 0
    if npoint == 0:
        return pcd
    idx = farthest_point_sample(torch.Tensor(pcd).t(), ratio=0, start=fps_start(seed, b, n), npoint=npoint)
    return pcd[idx.numpy()]


# --------------------------------------------------------------------------------------
# H4  transform: dataset/object.py:304-309 (inv=True -> object frame, "align_pc")
# --------------------------------------------------------------------------------------


def transform(pc: np.ndarray, R: np.ndarray, t: np.ndarray, inv: bool = False) -> np.ndarray:
    """`pc @ R + (-t @ R)` for inv, `pc @ R.T + t` otherwise; the 3-term dot products are
    evaluated left to right with separately rounded products (BLAS-order independent)."""
    pc = np.asarray(pc, dtype=np.float64)
    R = np.asarray(R, dtype=np.float64)
    t = np.asarray(t, dtype=np.float64).reshape(3)
    M = R if inv else R.T
    if inv:
        nt = -1.0 * t
        tt = np.array([(nt[0] * R[0, j] + nt[1] * R[1, j]) + nt[2] * R[2, j] for j in range(3)])
    else:
        tt = t
    out = np.empty_like(pc)
    for j in range(3):
        out[:, j] = ((pc[:, 0] * M[0, j] + pc[:, 1] * M[1, j]) + pc[:, 2] * M[2, j]) + tt[j]
    return out


# --------------------------------------------------------------------------------------
# H5  ball query: dataset/object.py:281-288 find_positives, :311-317 get_overlap
# --------------------------------------------------------------------------------------


def find_positives(pc1: np.ndarray, pc2: np.ndarray, r: float = 0.2) -> np.ndarray:
    distances = np.linalg.norm(pc1[:, np.newaxis] - pc2, axis=2)
    mask = distances <= r
    return np.argwhere(mask.astype(bool))


def find_positives_mask(pc1: np.ndarray, pc2: np.ndarray, r: float) -> np.ndarray:
    return np.linalg.norm(pc1[:, np.newaxis] - pc2, axis=2) <= r


def get_overlap(l_1: int, l_2: int, p: np.ndarray):
    overlap_12 = np.zeros((l_1), dtype=np.byte)
    overlap_21 = np.zeros((l_2), dtype=np.byte)
    overlap_12[p[:, 0]] = 1
    overlap_21[p[:, 1]] = 1
    return overlap_12, overlap_21


# --------------------------------------------------------------------------------------
# H6  batch assembly: dataset/helpers.py:22-50 collate
# --------------------------------------------------------------------------------------


def collate(data):
    """dataset/helpers.py:22-50 on a list of (CAD, PC, Obj) dicts: every ndarray field of
    CAD / PC becomes torch.Tensor (f32) padded by pad_sequence(batch_first=True), other CAD
    / PC fields None; Obj ndarray fields with more than one element are converted the same
    way and padded, except P which stays a list; everything else becomes a list."""
    def padded(key, part):
        return torch.nn.utils.rnn.pad_sequence([torch.Tensor(d[part][key]) for d in data], batch_first=True)

    CAD = {k: padded(k, 0) if isinstance(v, np.ndarray) else None for k, v in data[0][0].items()}
    PC = {k: padded(k, 1) if isinstance(v, np.ndarray) else None for k, v in data[0][1].items()}
    Obj = {}
    for k, v in data[0][2].items():
        if isinstance(v, np.ndarray) and v.size > 1:
            Obj[k] = [torch.Tensor(d[2][k]) for d in data] if k == "P" else padded(k, 2)
        else:
            Obj[k] = [d[2][k] for d in data]
    return CAD, PC, Obj


# --------------------------------------------------------------------------------------
# H10 / H11  fmap -> point map: fmap2pointmap_solvers/naive.py:6-34,
#            spacial_filtering.py:5-75
# --------------------------------------------------------------------------------------


def naive_nn_query(feat_x: torch.Tensor, feat_y: torch.Tensor, dim: int = -2) -> torch.Tensor:
    dist = torch.cdist(feat_x, feat_y)
    return dist.argmin(dim=dim)


def naive_fmap2pointmap(C12, evecs_x, evecs_y, **kwargs):
    if C12.dim() == 3:
        C12 = C12.squeeze(0)
    pp = naive_nn_query(torch.matmul(evecs_x, C12.t()), evecs_y)
    return torch.stack([pp, torch.linspace(0, pp.shape[0] - 1, pp.shape[0], device=pp.device).type(torch.int16)], 0)


def topk_nn_query(feat_x, feat_y, K: int = 5):
    """spacial_filtering.py:20-38 (sort along V1, first K rows per column, PC-major)."""
    dist = torch.cdist(feat_x, feat_y)
    _, idx = dist.sort(dim=-2, stable=True)
    idx = idx.t()[:, :K]
    idx_p = torch.linspace(0, idx.shape[0] - 1, idx.shape[0]).type(torch.int16).unsqueeze(1).repeat(1, K)
    return torch.stack([idx, idx_p], 0).reshape(2, -1)


def euclidean_distance(tensor):
    squared_distances = torch.sum((tensor[:, None] - tensor) ** 2, dim=2)
    return torch.sqrt(squared_distances)


def rigidity_scores(CAD, PC, p_pred):
    B = euclidean_distance(PC[p_pred[1]])
    A = euclidean_distance(CAD[p_pred[0]])
    return torch.absolute(A - B).mean(0)


def spacial_filtering(CAD, PC, p_pred, diam_cad, return_scores: bool = False):
    """spacial_filtering.py:51-75."""
    scores = []
    s = rigidity_scores(CAD, PC, p_pred)
    scores.append(s)
    p_pred = p_pred[:, s < 0.3 * diam_cad]
    s = rigidity_scores(CAD, PC, p_pred)
    scores.append(s)
    p_pred = p_pred[:, s < 0.15 * diam_cad]
    s = rigidity_scores(CAD, PC, p_pred)
    scores.append(s)
    if (s < 0.055 * diam_cad).sum() == 0:
        p_pred = p_pred[:, s < 0.065 * diam_cad]
    else:
        p_pred = p_pred[:, s < 0.055 * diam_cad]
    if return_scores:
        return p_pred, scores
    return p_pred


def spacial_filtering_fmap2pointmap(C12, evecs_x, evecs_y, CAD, PC, diam_cad):
    if C12.dim() == 3:
        C12 = C12.squeeze(0)
    pp = topk_nn_query(torch.matmul(evecs_x[:], C12.t()), evecs_y[:])
    return spacial_filtering(CAD, PC, pp, diam_cad)


# --------------------------------------------------------------------------------------
# H12  inlier ratio: utils/utils.py:81-105 ; H15 C_gt: utils/utils.py:67-79
# --------------------------------------------------------------------------------------


def compute_inlier_ratio(pred_corr, CAD, PC_aligned, threshold):
    total_corr = len(pred_corr)
    if total_corr == 0:
        return 0
    CAD = CAD[pred_corr[:, 0]]
    PC_aligned = PC_aligned[pred_corr[:, 1]]
    sq_dist = torch.square(CAD - PC_aligned).sum(-1) ** 0.5
    inliers = (sq_dist < (threshold)).sum()
    return inliers / total_corr


def C_from_sparse_P(P, evecs1, evecs2):
    evec_1_a, evec_2_a = evecs1[P[:, 0]], evecs2[P[:, 1]]
    return torch.linalg.lstsq(evec_2_a, evec_1_a)[0][:evec_1_a.size(-1)]


# --------------------------------------------------------------------------------------
# H13  RANSAC + Umeyama: scripts/test_RANSAC.py:288-310 -> Open3D 0.17
#      registration_ransac_based_on_correspondence + Eigen::umeyama (Appendix A).
#      Hypothesis index sets are inputs (Open3D's RNG is not reproducible).
# --------------------------------------------------------------------------------------


def umeyama(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """Eigen::umeyama(src[3,n], dst[3,n], with_scaling=false) -> 4x4."""
    n = src.shape[1]
    one_over_n = 1.0 / n
    src_mean = src.sum(axis=1) * one_over_n
    dst_mean = dst.sum(axis=1) * one_over_n
    src_demean = src - src_mean[:, None]
    dst_demean = dst - dst_mean[:, None]
    sigma = one_over_n * dst_demean @ src_demean.T
    U, S, Vt = np.linalg.svd(sigma)
    D = np.ones(3)
    if np.linalg.det(U) * np.linalg.det(Vt.T) < 0:
        D[2] = -1
    T = np.eye(4)
    T[:3, :3] = U @ np.diag(D) @ Vt
    T[:3, 3] = dst_mean - T[:3, :3] @ src_mean
    return T


def registration_icp(source: np.ndarray, target: np.ndarray, max_dist: float, init: np.ndarray,
                     max_iteration: int = 30, relative_fitness: float = 1e-6, relative_rmse: float = 1e-6):
    """scripts/test_RANSAC.py:436-446 -> Open3D 0.17 RegistrationICP with
    TransformationEstimationPointToPoint (parity unpinned: Open3D is absent). Per evaluation
    every source point T s takes its nearest target point (first index on exact ties; a KD-tree
    may return either), a pair iff d^2 < max_dist^2 (nanoflann's strict radius test);
    fitness = pairs / |source|, rmse = sqrt(sum d^2 / pairs). Update: umeyama of the pairs
    (identity without pairs), T <- U T; stop when |dfitness| < relative_fitness and
    |drmse| < relative_rmse. Returns (T, fitness, rmse, updates, converged)."""
    T = np.array(init, dtype=np.float64).reshape(4, 4)

    def evaluate(T):
        p = source @ T[:3, :3].T + T[:3, 3]
        d2 = ((p[:, None, :] - target[None, :, :]) ** 2).sum(-1)
        j = d2.argmin(1)
        best = d2[np.arange(len(p)), j]
        ok = best < max_dist * max_dist
        n = int(ok.sum())
        fit = n / len(p) if n else 0.0
        rmse = math.sqrt(best[ok].sum() / n) if n else 0.0
        return p[ok], target[j[ok]], fit, rmse

    P, Q, fit, rmse = evaluate(T)
    it, conv = 0, False
    while it < max_iteration:
        U = umeyama(P.T, Q.T) if len(P) else np.eye(4)
        T = U @ T
        pf, pr = fit, rmse
        P, Q, fit, rmse = evaluate(T)
        it += 1
        if abs(pf - fit) < relative_fitness and abs(pr - rmse) < relative_rmse:
            conv = True
            break
    return T, fit, rmse, it, conv


# ---------------------------------------------------------------------------- (f2) TEASER++
# scripts/test_teaser.py:327-331, 362-435 -> teaserpp_python RobustRegistrationSolver (absent:
# restated from the published TEASER++ algorithm, parity unpinned), estimate_scaling = False.


def teaser_graph(src: np.ndarray, dst: np.ndarray, beta: float) -> np.ndarray:
    """ScaleInliersSelector over all pairs: edge (i, j) iff ||a_j - a_i| - |b_j - b_i|| <= beta."""
    def norms(x):
        d = x[None, :, :] - x[:, None, :]
        return np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])
    e = np.abs(norms(src) - norms(dst)) <= beta
    np.fill_diagonal(e, False)
    return e


def core_numbers(adj: np.ndarray) -> np.ndarray:
    """k-core numbers by repeated minimum-degree peeling (pmc compute_cores)."""
    n = adj.shape[0]
    deg = adj.sum(1).astype(np.int64)
    alive = np.ones(n, bool)
    core = np.zeros(n, np.int64)
    k = 0
    for _ in range(n):
        cand = np.where(alive)[0]
        v = cand[np.argmin(deg[cand])]
        k = max(k, int(deg[v]))
        core[v] = k
        alive[v] = False
        deg[adj[v] & alive] -= 1
    return core


def max_clique_size(adj: np.ndarray) -> int:
    """Bron-Kerbosch with pivoting (exact; small graphs only)."""
    n = adj.shape[0]
    nb = [set(np.flatnonzero(adj[v])) for v in range(n)]
    best = [0]

    def bk(R, P, X):
        if not P and not X:
            best[0] = max(best[0], R)
            return
        if R + len(P) <= best[0]:
            return
        u = max(P | X, key=lambda w: len(P & nb[w]))
        for v in list(P - nb[u]):
            bk(R + 1, P & nb[v], X & nb[v])
            P = P - {v}
            X = X | {v}
    bk(0, set(range(n)), set())
    return best[0]


def svd_rot(X: np.ndarray, Y: np.ndarray, w: np.ndarray) -> np.ndarray:
    """teaser::utils::svdRot(X[3,m], Y[3,m], W): R = V U^T of H = X W Y^T, det-fixed."""
    H = (X * w[None, :]) @ Y.T
    U, _, Vt = np.linalg.svd(H)
    V = Vt.T
    if np.linalg.det(U) * np.linalg.det(V) < 0:
        V[:, 2] *= -1
    return V @ U.T


def gnc_tls_rotation(s: np.ndarray, d: np.ndarray, noise_bound: float, gnc_factor: float = 1.4,
                     max_iterations: int = 100, cost_threshold: float = 1e-12):
    """GNCTLSRotationSolver::solveForRotation on TIMs s, d [m, 3] -> (R, weights)."""
    m = s.shape[0]
    nb2 = noise_bound ** 2
    if nb2 < 1e-16:
        nb2 = 1e-2
    w = np.ones(m)
    mu, prev = 1.0, math.inf
    R = np.eye(3)
    for it in range(max_iterations):
        R = svd_rot(s.T, d.T, w)
        q = d - s @ R.T
        r2 = (q * q).sum(1)
        if it == 0:
            mu = 1.0 / (2.0 * r2.max() / nb2 - 1.0)
            if mu <= 0:
                break
        th1, th2 = (mu + 1) / mu * nb2, mu / (mu + 1) * nb2
        cost = float((w * r2).sum())
        w = np.where(r2 >= th1, 0.0, np.where(r2 <= th2, 1.0, np.sqrt(nb2 * mu * (mu + 1) / np.maximum(r2, 1e-300)) - mu))
        diff = abs(cost - prev)
        mu *= gnc_factor
        prev = cost
        if diff < cost_threshold:
            break
    return R, w


def scalar_tls(X: np.ndarray, rng: float):
    """ScalarTLSEstimator::estimate (adaptive voting) -> (estimate, inlier mask)."""
    N = X.shape[0]
    h = []
    for i in range(N):
        h.append((X[i] - rng, i + 1))
        h.append((X[i] + rng, -i - 1))
    h.sort(key=lambda p: p[0])  # stable
    w = 1.0 / (rng * rng)
    rsum, dxw, dw, sx, sx2, card = rng * N, 0.0, 0.0, 0.0, 0.0, 0
    best, est = math.inf, 0.0
    for val, sgn in h:
        i = abs(sgn) - 1
        e = 1 if sgn > 0 else -1
        card += e
        dw += e * w
        dxw += e * w * X[i]
        rsum -= e * rng
        sx += e * X[i]
        sx2 += e * X[i] * X[i]
        xh = dxw / dw
        cost = (card * xh * xh + sx2 - 2 * sx * xh) + rsum
        if cost < best:
            best, est = cost, xh
    return est, np.abs(X - est) <= rng


def teaser_from_clique(src: np.ndarray, dst: np.ndarray, clique, noise_bound=0.05, cbar2=1.0, gnc_factor=1.4,
                       max_iterations=100, cost_threshold=1e-12):
    """Steps 3-4 of RobustRegistrationSolver::solve given the sorted clique: chain TIMs, GNC-TLS
    (noise bound 2 noise), adaptive-voting translation over the clique -> (T, rot_inl, trans_inl)."""
    C = np.asarray(clique)
    m = C.size
    leaf = np.roll(C, -1)
    s, d = src[leaf] - src[C], dst[leaf] - dst[C]
    R, w = gnc_tls_rotation(s, d, 2 * noise_bound, gnc_factor, max_iterations, cost_threshold)
    raw = dst[C] - src[C] @ R.T
    t = np.zeros(3)
    inl = np.ones(m, bool)
    for r in range(3):
        t[r], ii = scalar_tls(raw[:, r], noise_bound * math.sqrt(cbar2))
        inl &= ii
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, t
    return T, int((w >= 0.5).sum()), int(inl.sum())


def ransac_evaluate(src: np.ndarray, dst: np.ndarray, corres: np.ndarray, T: np.ndarray, max_dist: float):
    """Open3D EvaluateRANSACBasedOnCorrespondence: fitness, inlier_rmse."""
    s = src[corres[:, 0]]
    p = (s @ T[:3, :3].T) + T[:3, 3]
    d = p - dst[corres[:, 1]]
    dis2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    inl = dis2 < max_dist * max_dist
    good = int(inl.sum())
    if good == 0:
        return 0.0, 0.0
    return good / corres.shape[0], math.sqrt(float(dis2[inl].sum()) / good)


def ransac_registration(src, dst, corres, hyps, max_dist=0.05):
    """Best hypothesis by (fitness desc, rmse asc, index asc). hyps: int [H,4] row ids into corres."""
    best = (-1.0, 0.0, -1, np.eye(4))
    if corres.shape[0] < 4 or max_dist <= 0:
        return np.eye(4), 0.0, 0.0, -1
    for h in range(hyps.shape[0]):
        c = corres[hyps[h]]
        T = umeyama(src[c[:, 0]].T, dst[c[:, 1]].T)
        f, r = ransac_evaluate(src, dst, corres, T, max_dist)
        if f > best[0] or (f == best[0] and r < best[1]):
            best = (f, r, h, T)
    return best[3], best[0], best[1], best[2]


# --------------------------------------------------------------------------------------
# H14  pose metrics: scripts/test_RANSAC.py:77-81, 154-238
# --------------------------------------------------------------------------------------


def pose_transform(pcd, pose):
    """test_RANSAC.py:154-160."""
    pcd_ = pcd @ pose[:3, :3].T
    return pcd_ + pose[:3:, -1]


def add(T_est, T_gt, pcd, diameter, percentage=0.1):
    """test_RANSAC.py:162-173."""
    pts_est = pose_transform(pcd, T_est)
    pts_gt = pose_transform(pcd, T_gt)
    e = np.linalg.norm(pts_est - pts_gt, axis=1).mean()
    return e, int(e < diameter * percentage)


def compute_add_score(pts3d, diameter, pose_gt, pose_pred, percentage=0.1):
    """test_RANSAC.py:186-201 (per-row "xyz direction" quirk, count = 3)."""
    R_gt, t_gt = pose_gt[:3, :3], pose_gt[:3, 3]
    R_pred, t_pred = pose_pred[:3, :3], pose_pred[:3, 3]
    count = R_gt.shape[0]
    mean_distances = np.zeros((count,), dtype=np.float32)
    for i in range(count):
        a = R_gt[i].reshape((1, 3)).dot(pts3d.transpose()) + t_gt[i]
        b = R_pred[i].reshape((1, 3)).dot(pts3d.transpose()) + t_pred[i]
        mean_distances[i] = np.mean(np.linalg.norm(a - b, axis=0))
    threshold = diameter * percentage
    return (mean_distances < threshold).sum() / count


def compute_adds_score(pts3d, diameter, pose_gt, pose_pred, percentage=0.1):
    """test_RANSAC.py:203-222 — 1-NN (KDTree) on the per-row 1-D projections."""
    R_gt, t_gt = pose_gt[:3, :3], pose_gt[:3, 3]
    R_pred, t_pred = pose_pred[:3, :3], pose_pred[:3, 3]
    count = R_gt.shape[0]
    mean_distances = np.zeros((count,), dtype=np.float32)
    for i in range(count):
        if np.isnan(np.sum(t_pred[i])):
            mean_distances[i] = np.inf
            continue
        a = (R_gt[i].reshape((1, 3)).dot(pts3d.transpose()) + t_gt[i]).ravel()
        b = (R_pred[i].reshape((1, 3)).dot(pts3d.transpose()) + t_pred[i]).ravel()
        sa = np.sort(a)
        pos = np.clip(np.searchsorted(sa, b), 1, len(sa) - 1)
        d0 = b - sa[pos - 1]
        d1 = sa[pos] - b
        # sklearn KDTree reports sqrt(rdist) with rdist = d*d
        d = np.minimum(np.sqrt(d0 * d0), np.sqrt(d1 * d1))
        mean_distances[i] = np.mean(d)
    threshold = diameter * percentage
    return (mean_distances < threshold).sum() / count


def get_angular_error(R_exp, R_est):
    """test_RANSAC.py:77-81."""
    return abs(np.arccos(min(max(((np.matmul(R_exp.T, R_est)).trace() - 1) / 2, -1.0), 1.0)))
