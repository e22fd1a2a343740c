"""(f2) TEASER++ host stages (pk_teaser_solve: k-core / max clique, GNC-TLS rotation, adaptive
voting) against the numpy restatement in oracle/dpfm_oracle.py, on host inputs — no GPU needed:
the consistency graph comes from the oracle (its device twin is tested in test_teaser_gpu.py).

  * dense inlier sets (the k-core heuristic path): the clique is the oracle's max k-core exactly;
  * sparse inlier sets (the exact path): the clique is a clique of the oracle's maximum size;
  * given that clique, T within 1e-9 of the oracle's GNC-TLS + adaptive voting, same rotation
    and translation inlier counts; the recovered pose is the planted one;
  * degenerate crops (0, 1, 2 correspondences, no consistent pair): invalid, identity.
"""
import numpy as np
import pytest

from oracle import dpfm_oracle as O


def pack_bits(adj: np.ndarray, nmax: int) -> np.ndarray:
    n = adj.shape[0]
    W = (nmax + 63) // 64
    full = np.zeros((nmax, W * 64), bool)
    full[:n, :n] = adj
    return np.packbits(full.reshape(nmax, W * 64), axis=1, bitorder="little").view(np.uint64).reshape(nmax, W)


def planted(rng, n, inlier_frac, noise=0.01):
    from dpfm_amd.dataset.synthetic import random_rotation
    R = random_rotation(rng)
    t = rng.normal(size=3) * 10 + np.array([0, 0, 80.0])
    a = rng.normal(size=(n, 3)) * 5
    b = a @ R.T + t + rng.normal(size=(n, 3)) * noise
    out = rng.random(n) >= inlier_frac
    b[out] = rng.normal(size=(out.sum(), 3)) * 5 + t
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, t
    return a, b, T


def run_host(crops, nmax, **kw):
    from dpfm_amd import _lib, ops
    p = _lib.TeaserParams(kw.get("noise_bound", 0.05), 1.0, 1.4, 1e-12, 0.5, 100, 0, kw.get("budget", 2_000_000))
    a = np.concatenate([c[0] for c in crops] + [np.zeros((1, 3))])
    b = np.concatenate([c[1] for c in crops] + [np.zeros((1, 3))])
    off = np.concatenate([[0], np.cumsum([c[0].shape[0] for c in crops])]).astype(np.int64)
    adj = np.stack([pack_bits(O.teaser_graph(c[0], c[1], 0.1) if c[0].shape[0] else np.zeros((0, 0), bool), nmax)
                    for c in crops])
    deg = np.stack([np.pad(O.teaser_graph(c[0], c[1], 0.1).sum(1), (0, nmax - c[0].shape[0])) if c[0].shape[0]
                    else np.zeros(nmax, np.int64) for c in crops]).astype(np.int32)
    return ops.teaser_solve_host(a, b, off, nmax, adj, deg, p, threads=4)


@pytest.mark.parametrize("frac,n,mode", [(0.8, 150, 2), (0.3, 70, 1), (0.15, 90, 1)])
def test_teaser_host_matches_oracle(frac, n, mode):
    rng = np.random.default_rng(int(frac * 100) + n)
    crops = [planted(rng, n - 7 * k, frac) for k in range(3)]
    nmax = n
    T, clique, size, info = run_host(crops, nmax)
    for k, (a, b, Tt) in enumerate(crops):
        adj = O.teaser_graph(a, b, 0.1)
        C = clique[k, :size[k]]
        assert info[k, 0] == 1 and info[k, 1] == mode, info[k]
        if mode == 2:
            core = O.core_numbers(adj)
            np.testing.assert_array_equal(C, np.flatnonzero(core >= core.max()))
        else:
            assert size[k] == O.max_clique_size(adj)
            sub = adj[np.ix_(C, C)]
            assert (sub | np.eye(len(C), dtype=bool)).all()
        To, rin, tin = O.teaser_from_clique(a, b, C)
        np.testing.assert_allclose(T[k], To, atol=1e-9)
        assert info[k, 2] == rin and info[k, 3] == tin
        assert np.abs(T[k][:3, :3] - Tt[:3, :3]).max() < 5e-3 and np.abs(T[k][:3, 3] - Tt[:3, 3]).max() < 0.05


def test_teaser_host_degenerate():
    rng = np.random.default_rng(1)
    far = (rng.normal(size=(5, 3)) * 100, rng.normal(size=(5, 3)) * 0.001)  # no consistent pair
    crops = [(np.zeros((0, 3)), np.zeros((0, 3))), (np.ones((1, 3)), np.ones((1, 3))),
             (np.eye(3)[:2] * 3, np.eye(3)[:2] * 3), far]
    T, clique, size, info = run_host(crops, 8)
    for k in (0, 1, 3):
        assert info[k, 0] == 0 and np.array_equal(T[k], np.eye(4)), (k, info[k])
    assert size[2] == 2 and info[2, 0] == 1  # a consistent pair: a valid (degenerate) fit
