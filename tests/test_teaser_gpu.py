"""(f2) TEASER++ on the device: pk_teaser_graph's consistency bitsets bit-exact against the
numpy restatement (oracle/dpfm_oracle.py teaser_graph) on ragged crops, including padding rows
and empty crops; end to end (ops.teaser = device graph + host solve) against the host-only path
fed with the oracle's graph (tests/test_teaser_cpu.py pins that path against the oracle), and the
reference-shaped RobustRegistrationSolver interface."""
import numpy as np
import pytest
import torch

from oracle import dpfm_oracle as O
from test_teaser_cpu import pack_bits, planted, run_host

pytestmark = pytest.mark.gpu


def _pack(crops, device):
    a = np.concatenate([c[0] for c in crops] + [np.zeros((1, 3))])
    b = np.concatenate([c[1] for c in crops] + [np.zeros((1, 3))])
    off = np.concatenate([[0], np.cumsum([c[0].shape[0] for c in crops])]).astype(np.int64)
    return (torch.from_numpy(a).to(device), torch.from_numpy(b).to(device), torch.from_numpy(off).to(device))


def test_teaser_graph_bitexact(device):
    from dpfm_amd import ops
    rng = np.random.default_rng(0)
    crops = [planted(rng, n, 0.4) for n in (300, 0, 129, 64, 1, 257)]
    nmax = 300
    a, b, off = _pack(crops, device)
    adj, deg = ops.teaser_graph(a, b, off, nmax, 0.1)
    adj = adj.cpu().numpy().view(np.uint64)
    deg = deg.cpu().numpy()
    for k, (ca, cb, _) in enumerate(crops):
        ref = O.teaser_graph(ca, cb, 0.1) if ca.shape[0] else np.zeros((0, 0), bool)
        np.testing.assert_array_equal(adj[k], pack_bits(ref, nmax), err_msg=f"crop {k}")
        np.testing.assert_array_equal(deg[k, :ca.shape[0]], ref.sum(1))
        assert (deg[k, ca.shape[0]:] == 0).all()


def test_teaser_end_to_end_matches_host_path(device):
    from dpfm_amd import ops
    rng = np.random.default_rng(3)
    crops = [planted(rng, n, f) for n, f in ((400, 0.8), (150, 0.3), (90, 0.15), (2, 1.0), (0, 1.0))]
    nmax = 400
    a, b, off = _pack(crops, device)
    got = ops.teaser(a, b, off, nmax, threads=4)
    ref = run_host(crops, nmax)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)


def test_robust_registration_solver_interface(device):
    from dpfm_amd.pose.teaser import RobustRegistrationSolver
    rng = np.random.default_rng(5)
    a, b, Tt = planted(rng, 500, 0.5)
    p = RobustRegistrationSolver.Params()
    p.cbar2, p.noise_bound, p.estimate_scaling = 1, 0.05, False
    p.rotation_gnc_factor, p.rotation_max_iterations, p.rotation_cost_threshold = 1.4, 100, 1e-12
    solver = RobustRegistrationSolver(p, device=device)
    solver.solve(a.T, b.T)
    sol = solver.getSolution()
    assert sol.valid and sol.scale == 1.0
    assert np.abs(sol.rotation - Tt[:3, :3]).max() < 5e-3 and np.abs(sol.translation - Tt[:3, 3]).max() < 0.05
