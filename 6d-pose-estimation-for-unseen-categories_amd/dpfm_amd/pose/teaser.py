"""TEASER++ pose solver — the (f2) row: scripts/test_teaser.py:327-331, 362-435 builds
`teaserpp_python.RobustRegistrationSolver(params)` with cbar2 = 1, noise_bound = 0.05,
estimate_scaling = False, GNC_TLS rotation (gnc factor 1.4, 100 iterations, cost threshold
1e-12) and calls `solver.solve(src[3,n], dst[3,n])`, `solver.getSolution()` (.rotation,
.translation, .valid).

`RobustRegistrationSolver` keeps that interface; `teaser_batched` solves many crops at once.
The pairwise-consistency graph (O(n^2)) is built on the device (csrc/teaser.hip); the clique
search, GNC-TLS and adaptive voting run as native host code (parity unpinned: the TEASER++
package is absent, restated from its published algorithm)."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops


@dataclass
class TeaserSolution:
    """The fields of teaser::RegistrationSolution the reference reads, plus the clique."""
    valid: bool
    scale: float
    rotation: np.ndarray
    translation: np.ndarray
    max_clique: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    clique_mode: str = "exact"  # exact | budget | kcore
    rotation_inliers: int = 0
    translation_inliers: int = 0


class RobustRegistrationSolver:
    """teaserpp_python.RobustRegistrationSolver with the reference's parameter fields."""

    class Params:
        def __init__(self):
            self.cbar2 = 1.0
            self.noise_bound = 0.01
            self.estimate_scaling = True
            self.rotation_gnc_factor = 1.4
            self.rotation_max_iterations = 100
            self.rotation_cost_threshold = 1e-6
            self.kcore_heuristic_threshold = 0.5
            self.max_clique_nodes = 2_000_000

    def __init__(self, params: "RobustRegistrationSolver.Params", device=None):
        if params.estimate_scaling:
            raise NotImplementedError("estimate_scaling=True is not supported (the reference sets it False)")
        self.params = params
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._sol = None

    def solve(self, src, dst):
        """src, dst: [3, n] (TEASER's column convention)."""
        a = torch.as_tensor(np.asarray(src, dtype=np.float64).T.copy(), device=self.device)
        b = torch.as_tensor(np.asarray(dst, dtype=np.float64).T.copy(), device=self.device)
        off = torch.tensor([0, a.shape[0]], dtype=torch.int64, device=self.device)
        p = self.params
        T, clique, size, info = ops.teaser(a, b, off, a.shape[0], p.noise_bound, p.cbar2, p.rotation_gnc_factor,
                                           p.rotation_max_iterations, p.rotation_cost_threshold,
                                           p.kcore_heuristic_threshold, p.max_clique_nodes, threads=1)
        self._sol = _solution(T[0], clique[0], size[0], info[0])
        return self._sol

    def getSolution(self) -> TeaserSolution:  # noqa: N802 (reference API name)
        return self._sol


def _solution(T, clique, size, info) -> TeaserSolution:
    mode = {1: "exact", 0: "budget", 2: "kcore"}[int(info[1])]
    return TeaserSolution(bool(info[0]), 1.0, T[:3, :3].copy(), T[:3, 3].copy(), clique[:int(size)].copy(), mode,
                          int(info[2]), int(info[3]))


def teaser_batched(src, dst, off, nmax=None, threads: int = 8, **params):
    """Device tensors (matched pairs packed by off) -> list of TeaserSolution, one per crop."""
    T, clique, size, info = ops.teaser(src, dst, off, nmax, threads=threads, **params)
    return [_solution(T[b], clique[b], size[b], info[b]) for b in range(T.shape[0])]
