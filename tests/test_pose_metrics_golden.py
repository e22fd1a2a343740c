"""CPU: the H14 metric restatements reproduce the reference's own published per-crop
outputs (results_on_*/results_poses_RANSAC — golden vectors minted by
tests/golden/make_golden.py). This is the oracle's pin for the pose metrics."""
import os

import numpy as np
import pytest

from oracle import dpfm_oracle as O

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "pose_metrics.npz"))
N = int(G["n"])


@pytest.mark.parametrize("k", range(N))
def test_reference_pose_metrics(k):
    cad = G[f"{k}_cad"]
    T_gt, T_icp, T_pred = G[f"{k}_T_gt_full"], G[f"{k}_T_icp_full"], G[f"{k}_T_pred"]
    diam = float(G[f"{k}_diam"])
    # "Avg. Euclidean Distance (ADD) ICP" (test_RANSAC.py:453) from full-precision poses
    e, _ = O.add(T_icp, T_gt, cad, diam)
    np.testing.assert_allclose(e, float(G[f"{k}_add_icp"]), rtol=1e-9)
    # "Avg. Euclidean Distance (ADD) [cm]" (pre-ICP; T_pred is only printed to 9 digits)
    e0, _ = O.add(T_pred, T_gt, cad, diam)
    np.testing.assert_allclose(e0, float(G[f"{k}_add"]), rtol=2e-5, atol=1e-5)
    # "Add Score ICP thres (xyz direction)" (compute_add_score quirk, :461)
    assert O.compute_add_score(cad, diam, T_gt, T_icp) == float(G[f"{k}_add_xyz_icp"])
    # "Add-S Score ICP" (compute_adds_score, :466)
    assert O.compute_adds_score(cad, diam, T_gt, T_icp) == float(G[f"{k}_adds_icp"])
    # "Error [cm]" / "Error [deg]" (:474-477)
    np.testing.assert_allclose(np.linalg.norm(T_gt[:3, 3] - T_icp[:3, 3]), float(G[f"{k}_err_cm"]), rtol=1e-9)
    deg = O.get_angular_error(T_gt[:3, :3], T_icp[:3, :3]) * 180 / np.pi
    np.testing.assert_allclose(deg, float(G[f"{k}_err_deg"]), rtol=1e-6, atol=1e-6)
