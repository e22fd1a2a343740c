"""dpfm_amd — MI355X-native drop-in for the RGB-D pose-inference hot path of
m13ammed/6D-Pose-Estimation-for-Unseen-Categories.

Module layout mirrors the reference so call sites read the same:
  dataset/object.py, dataset/helpers.py   crop formation, ball query, collate
  models/dpfm.py, modeling/dpfm.py        DPFMNet and its refinement / fmap heads
  fmap2pointmap_solvers/                  naive + spatial-filtering point-map solvers
  utils/utils.py, utils/loss.py           C_from_sparse_P, inlier ratio, DPFMLoss
  pose/                                   RANSAC + Umeyama pose fit, ADD metrics
  dpfm_utils.py                           upstream DPFM helpers (FPS, get_mask, WBCE)
  ops.py                                  torch front-ends of libposekern.so (C-ABI)
"""
__version__ = "0.1.0"
