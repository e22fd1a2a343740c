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

import os as _os

# ROCm 7.2 CLR pre-records the AQL packets of a captured HIP graph ("graph packet
# capture"); memset nodes recorded that way run on the first launch only and are skipped
# on every later replay (tools/memset_graph_probe.py: 19/20 replays wrong, 0/20 with it
# off). The training step is replayed as a graph and torch's own kernels issue memsets
# (split-reduction semaphores), so packet capture is switched off. This must happen
# before the HIP runtime initialises: import dpfm_amd before the first GPU call (bench.py,
# __graft_entry__.py and tests/conftest.py also set it first thing).
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
