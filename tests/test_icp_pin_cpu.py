"""The ICP oracle (oracle/c/oracle.c oc_icp) pinned by the reference's own Open3D outputs.

tests/golden/icp_pin.npz (minted by tests/golden/make_golden.py from the reference's
results_on_*/results_poses_* plys and txts) holds, per published crop, T_gt, the solver's
pose as printed (the ICP init) and the reference's ICP result T_pred_ICP. test_RANSAC.py:424-446
runs registration_icp(source = CAD, target = transform(CAD, T_gt), 0.2, T_est, PointToPoint,
max_iteration = 2000); the oracle rerun from the printed init lands within 1e-6 of the
reference's output on all 512 crops (max 3.9e-7, the 9-digit print of the init itself on a
crop with no pair inside the radius). This CPU test reruns a spread of crops that converge in
few iterations (the brute-force oracle costs ~60 ms per evaluation on 5000 x 5000 points);
tests/test_icp_gpu.py::test_icp_pinned_by_reference_outputs runs all 512 through pk_icp.
"""
import ctypes
import os

import numpy as np
import pytest

from _util import cp

GOLD = os.path.join(os.path.dirname(__file__), "golden")
# crops of all four result directories and all five objects, 1 - 15 ICP updates each; 40 has
# fitness 0.8 (converges onto the GT-posed CAD), 437 has no pair inside the radius
CROPS = (37, 40, 71, 87, 101, 178, 231, 362, 414, 437, 142, 15)


@pytest.fixture(scope="module")
def pin():
    g = dict(np.load(os.path.join(GOLD, "icp_pin.npz")))
    rc = np.load(os.path.join(GOLD, "real_crops.npz"))
    cads = {int(o): np.ascontiguousarray(rc[f"cad_{int(o)}"]) for o in np.unique(g["obj_id"])}
    return g, cads


def test_icp_pin_fixture_consistent(pin):
    g, cads = pin
    n = g["obj_id"].shape[0]
    assert n == 512 and set(cads) == {5, 6, 8, 11, 12}
    assert set(np.unique(g["tree"] * 2 + g["solver"]).tolist()) == {0, 1, 2, 3}
    assert (g["target_dev"] <= 1e-12).all()  # transform(CAD, T_gt) reproduces the target ply
    # the data as the reference holds it: the real-capture GT rotations are orthonormal only to
    # ~1e-2 (results_on_real; the PBR ones to ~1e-6, json precision), and three TEASER poses of results_on_pbr are degenerate; ICP
    # takes them as they are (an affine target, a non-rigid init), and so do the tests
    R = g["T_gt"][:, :3, :3]
    orth = np.abs(np.einsum("nij,nkj->nik", R, R) - np.eye(3)).reshape(n, -1).max(1)
    assert orth[g["tree"] == 0].max() < 2e-6 and orth.max() < 2e-2


def test_oracle_icp_matches_reference_outputs(coracle, pin):
    g, cads = pin
    for k in CROPS:
        cad = cads[int(g["obj_id"][k])]
        Tg = g["T_gt"][k]
        tgt = np.ascontiguousarray(cad @ Tg[:3, :3].T + Tg[:3, 3])  # test_RANSAC.py:154-160
        T0 = np.ascontiguousarray(g["T_pred"][k])
        T, st = np.zeros(16), np.zeros(4)
        coracle.oc_icp(cp(cad), cad.shape[0], cp(tgt), tgt.shape[0], cp(T0), 0.2, 2000, 1e-6, 1e-6, cp(T), cp(st))
        assert st[3] == 1, (k, st)
        err = np.abs(T.reshape(4, 4) - g["T_icp"][k]).max()
        assert err <= 1e-6, (k, err, st)
